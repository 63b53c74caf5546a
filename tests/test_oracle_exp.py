"""The oracle's vd_expf against the reference's own torch.exp / softmax (CPU).

The oracle and the device twin evaluate the decode exp (utils_bbox.py:52) and the
softmax exp (retinaface.py:147) with vd_expf (oracle/vdexp.py), so "post-processing
bit-exact" is exact against that shared function. These tests measure what the
substitution changes against torch's own exp: on the oracle's torch-CPU fp32 heads
(the reference's forward arithmetic) the keep lists and int boxes are replayed with
torch.exp in decode and softmax (oracle/bbox.py scores_boxes, forms "divide" and
"torch") and every frame that changes must be explained (tests/fp32_parity.explain)
as a decision within the exp's own rounding of its threshold. Full measurement over
every parity case: tools/exp_substitution.py -> profiles/r05_exp_substitution.json
(0 of 232 frames changed).
"""
import numpy as np
import pytest
import torch

import fp32_parity as fp
from conftest import face_weights


def test_vd_expf_within_one_ulp_of_torch_exp():
    from oracle.vdexp import vd_expf
    rng = np.random.default_rng(5)
    x = np.concatenate([rng.normal(0, 4, 400000), rng.uniform(-87, 88, 200000),
                        np.linspace(-20, 20, 100001)]).astype(np.float32)
    a = vd_expf(x).view(np.int32).astype(np.int64)
    b = torch.exp(torch.from_numpy(x)).numpy().view(np.int32).astype(np.int64)
    d = np.abs(a - b)
    assert d.max() <= 1
    assert d.mean() < 0.02          # torch's SLEEF exp is off the correctly rounded value ~1 % of the time


@pytest.mark.parametrize("form", ["divide", "torch"])
def test_exp_substitution_changes_no_c1_frame(form):
    """C1 (16 synthetic 640x640 frames, seeded R50): torch's exp changes no keep list
    or int box; if a frame did change, its first differing decision must straddle its
    threshold by less than the two exps' own difference (the explain record)."""
    from oracle import anchors, letterbox
    from oracle.retinaface import build_oracle_model
    from vdmi import synth
    frames = synth.frames(16, 640, 640, seed=0)
    m = build_oracle_model(face_weights("default"))
    pri = anchors.get_anchors((640, 640))
    changed, faces = [], 0
    for s in range(0, 16, 8):
        x, _ = letterbox.preprocess(list(frames[s:s + 8]))
        with torch.no_grad():
            loc, cls, _ = m.forward_raw(torch.from_numpy(x))
        for j in range(loc.shape[0]):
            faces += len(fp.frame_result(loc[j].numpy(), cls[j].numpy(), pri, 640, 640)[0])
            e = fp.explain(loc[j].numpy(), cls[j].numpy(), loc[j].numpy(), cls[j].numpy(), pri, 640, 640,
                           exp_o=None, exp_g=form)
            if e is not None:
                changed.append(e)
    assert faces > 100
    for e in changed:
        assert e["dist"] <= e["delta"] and e["dist_gpu"] <= e["delta"], e
        assert e["delta"] <= {"score": 3e-7, "order": 3e-7, "iou": 3e-7, "trunc": 1e-4}[e["kind"]], e
    assert len(changed) == 0, changed      # measured: 0 / 16 (profiles/r05_exp_substitution.json)
