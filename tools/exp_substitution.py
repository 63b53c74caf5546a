"""How much does the oracle's shared vd_expf change the reference's boxes?

The oracle (and the device twin in csrc/vd_math.h) evaluates the decode exp
(utils_bbox.py:52) and the softmax exp (retinaface.py:147) with vd_expf, a
fully specified, correctly rounded double evaluation; the reference calls
torch.exp / F.softmax. This replays the oracle's post-processing on the oracle's
own torch-CPU fp32 heads (the reference's forward arithmetic) for every frame of
the fp32 parity cases (tests/test_gpu_parity_fp32.py CASES, R50 seeded weights; plus
MobileNet-0.25 at C3 and the "dense" R50 weights -- thousands of candidates per
frame -- at C1)
three ways and counts frames whose keep lists or int boxes change:

  divide  torch.exp in decode and in the softmax, softmax as max / exp / e_k / sum
          (the form torch's CUDA softmax takes for 2-wide rows: where the reference
          runs, its CPU path raises at utils_bbox.py's .cuda());
  torch   torch.exp in decode, torch.softmax on the CPU as-is (multiplies by 1/sum).

Every changed frame is explained with tests/fp32_parity.explain (the first decision
that differs and how far it sits from its threshold).

    python tools/exp_substitution.py [out.json] [--cases c1_640_b16,...]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "video-desensitization_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402


def measure(case, frames, sd, forms=("divide", "torch"), chunk=8):
    import torch
    import fp32_parity as fp
    from oracle import anchors, letterbox
    from oracle.retinaface import build_oracle_model
    from oracle.vdexp import vd_expf
    m = build_oracle_model(sd)
    pri = anchors.get_anchors((640, 640))
    n, h, w = frames.shape[:3]
    rec = {"case": case, "frames": n, "faces": 0, "exp_args": 0, "exp_ulp_diff": {}}
    for f in forms:
        rec[f] = {"changed_frames": 0, "explained": []}
    diffs = {0: 0, 1: 0, 2: 0}
    for s in range(0, n, chunk):
        x, _ = letterbox.preprocess(list(frames[s:s + chunk]))
        with torch.no_grad():
            loc, cls, _ = m.forward_raw(torch.from_numpy(x))
        loc, cls = loc.numpy(), cls.numpy()
        for j in range(loc.shape[0]):
            b = s + j
            idx, _, _ = fp.frame_result(loc[j], cls[j], pri, h, w)
            rec["faces"] += len(idx)
            # exp arguments of the frame: loc_wh * 0.2 and the softmax logit differences
            c = cls[j]
            mx = np.maximum(c[:, 0], c[:, 1])
            args = np.concatenate([(loc[j][:, 2:] * np.float32(0.2)).ravel(), c[:, 0] - mx, c[:, 1] - mx])
            e1 = vd_expf(args).view(np.int32).astype(np.int64)
            e2 = torch.exp(torch.from_numpy(args)).numpy().view(np.int32).astype(np.int64)
            for k, v in zip(*np.unique(np.minimum(np.abs(e1 - e2), 2), return_counts=True)):
                diffs[int(k)] += int(v)
            rec["exp_args"] += args.size
            for f in forms:
                e = fp.explain(loc[j], cls[j], loc[j], cls[j], pri, h, w, exp_o=None, exp_g=f)
                if e is not None:
                    e["frame"] = b
                    rec[f]["changed_frames"] += 1
                    rec[f]["explained"].append(e)
    rec["exp_ulp_diff"] = {"0": diffs[0], "1": diffs[1], ">=2": diffs[2]}
    return rec


def cases():
    from test_gpu_parity_fp32 import CASES
    return CASES


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    sel = None
    for a in sys.argv[1:]:
        if a.startswith("--cases="):
            sel = a.split("=", 1)[1].split(",")
    out = args[0] if args else os.path.join(ROOT, "profiles", "r05_exp_substitution.json")
    from conftest import face_weights
    res = {"what": __doc__.split("\n\n")[1].replace("\n", " "), "cases": []}
    t0 = time.time()
    runs = [(c, "default") for c in cases()] + [("c3_1080p_b64", "mnet"), ("c1_640_b16", "dense")]
    for case, wkind in runs:
        if sel and case not in sel:
            continue
        r = measure(case, cases()[case](), face_weights(wkind))
        r["weights"] = wkind
        print(json.dumps({k: (v if k not in ("divide", "torch") else {"changed_frames": v["changed_frames"]})
                          for k, v in r.items()}), flush=True)
        res["cases"].append(r)
    res["seconds"] = round(time.time() - t0, 1)
    with open(out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
