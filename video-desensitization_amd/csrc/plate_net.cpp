// plate_net.cpp — YOLOv8n plate detector (placeholder until the plan lands).
#include "nets.h"

int vd_build_plate(Ctx& ctx, const WMap& W) {
    (void)ctx; (void)W;
    return vd_set_error(VD_ERR_STATE, "YOLOv8n plan not built in this version");
}
int vd_plate_forward(Ctx& ctx, const uint8_t* d, int n, int h, int w, size_t pitch) {
    (void)ctx; (void)d; (void)n; (void)h; (void)w; (void)pitch;
    return vd_set_error(VD_ERR_STATE, "YOLOv8n not available");
}
int vd_plate_post(Ctx& ctx, int n, int img_h, int img_w, const BoxTargets& t) {
    (void)ctx; (void)n; (void)img_h; (void)img_w; (void)t;
    return vd_set_error(VD_ERR_STATE, "YOLOv8n not available");
}

extern "C" int vdt_plate_raw(vd_ctx* h, const uint8_t* frames, int n, int fh, int fw, size_t pitch, int where,
                             float* out, int* anchors) {
    (void)h; (void)frames; (void)n; (void)fh; (void)fw; (void)pitch; (void)where; (void)out; (void)anchors;
    return vd_set_error(VD_ERR_STATE, "YOLOv8n not available");
}
