"""vd_jpeg_decode on the GPU: bit-exact against Pillow's libjpeg-turbo (and the
oracle) for every supported layout, batched 1080p frames decoded straight into
device memory, and those frames through vd_process identical to host-decoded ones."""
import io

import numpy as np
import pytest
from PIL import Image

from test_jpeg import CASES, make_jpeg, pillow_rgb

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def jctx(gpu):
    import vdmi
    from vdmi import weights
    ctx = vdmi.Context(precision="fp32", max_batch=8)
    ctx.load_weights(0, weights.retinaface_state_dict(0))
    yield ctx
    ctx.close()


@pytest.mark.parametrize("case", CASES + [(40, 56, 90, 2, 0, 3)])
def test_decode_matches_pillow(jctx, case):
    h, w, q, sub = case[:4]
    d = make_jpeg(h, w, q, sub, restart=case[5] if len(case) > 5 else None)
    got = jctx.jpeg_decode([d, d])
    exp = pillow_rgb(d)
    np.testing.assert_array_equal(got[0], exp)
    np.testing.assert_array_equal(got[1], exp)


def _video_frames(n, h=1080, w=1920, q=95):
    """ffmpeg-like frames: synthetic 1080p RGB encoded by libjpeg (Pillow) at q95, 4:2:0."""
    from vdmi import synth
    fr = synth.frames(n, h, w, seed=5)
    out = []
    for f in fr:
        b = io.BytesIO()
        Image.fromarray(f).save(b, "JPEG", quality=q)
        out.append(b.getvalue())
    return out


def test_batch_1080p_device_decode_and_process(jctx):
    import torch
    from vdmi import _lib
    jp = _video_frames(6)
    dev = torch.device("cuda:0")
    d = torch.empty((6, 1080, 1920, 3), dtype=torch.uint8, device=dev)
    jctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    try:
        jctx.jpeg_decode(jp, out=d)
        torch.cuda.synchronize()
        host = np.stack([pillow_rgb(j) for j in jp])
        np.testing.assert_array_equal(d.cpu().numpy(), host)
        # decoded-on-device frames through the hot path == host-decoded frames
        out_d, faces_d, _ = jctx.process(d)
        torch.cuda.synchronize()
        lists_d = jctx.read_boxes(_lib.VD_NET_RETINAFACE, 6)
        out_h, faces_h, _ = jctx.process(host)
        lists_h = jctx.read_boxes(_lib.VD_NET_RETINAFACE, 6)
        np.testing.assert_array_equal(out_d.cpu().numpy(), out_h)
        np.testing.assert_array_equal(lists_d.count, lists_h.count)
        for b in range(6):
            np.testing.assert_array_equal(lists_d.frame(b)[0], lists_h.frame(b)[0])
    finally:
        jctx.set_stream(None)
