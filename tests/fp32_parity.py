"""Box-parity bookkeeping for the fp32 plans (test infrastructure).

The reference's box indices come from its fp32 forward (face.py:133) followed by
decode / score >= 0.5 / greedy NMS at IoU 0.4 / box correction / int()
(utils_bbox.py:103-130, :12-43, face.py:139-148, combine_detect.py:243). Two fp32
forwards that sum the same products in different orders (torch-CPU vs MFMA tiles)
agree to f32 rounding, so a decision that sits closer to its threshold than that
rounding can flip. This module compares a GPU frame with the oracle frame and,
when they differ, names the FIRST decision that differs and measures how far it
sits from its threshold on both sides:

* ``score``   an anchor is a candidate on one side only (score vs 0.5, inclusive);
* ``order``   the same candidates sort differently (two scores tie within rounding);
* ``iou``     the same candidate is suppressed on one side only (IoU vs 0.4);
* ``trunc``   identical keep lists, an int() of a box coordinate differs (the
              float coordinate straddles an integer).

Every comparison first replays the oracle's post-processing on the GPU's own head
outputs and requires the GPU's keep list and int boxes exactly (post-processing is
bit-exact given the heads), so the only thing left to explain is the forward's
rounding.
"""
import numpy as np

from oracle import bbox as obbox

F32 = np.float32


def _iou(b, i, j):
    """torchvision nms ratio in float32 for boxes b[i], b[j] (oracle/bbox.py)."""
    bi, bj = b[i].astype(F32), b[j].astype(F32)
    ai = (bi[2] - bi[0]) * (bi[3] - bi[1])
    aj = (bj[2] - bj[0]) * (bj[3] - bj[1])
    w = max(F32(0), min(bi[2], bj[2]) - max(bi[0], bj[0]))
    h = max(F32(0), min(bi[3], bj[3]) - max(bi[1], bj[1]))
    inter = F32(w * h)
    return float(F32(inter / F32(F32(ai + aj) - inter)))


def nms_log(boxes, score, thr=0.5, iou=0.4):
    """Greedy NMS (torchvision semantics) with its decisions: returns (order of
    candidates, {candidate: suppressor or -1})."""
    cand = np.nonzero(score >= F32(thr))[0]
    order = cand[np.argsort(-score[cand], kind="stable")]
    kept, by = [], {}
    for c in order:
        sup = -1
        for k in kept:
            if _iou(boxes, k, c) > iou:
                sup = k
                break
        by[int(c)] = sup
        if sup < 0:
            kept.append(int(c))
    return order, by


def frame_result(loc, conf, pri, h, w, torch_exp=None):
    idx, boxes, _ = obbox.postprocess_frame(loc, conf, pri, 0.5, 0.4, torch_exp=torch_exp)
    fb = obbox.correct_and_scale(boxes, h, w)
    return idx, obbox.truncate_boxes(fb), fb


def explain(oloc, oconf, gloc, gconf, pri, h, w, exp_o=None, exp_g=None):
    """First differing decision between oracle heads (o) and GPU heads (g) of one
    frame, or None if keep lists and int boxes agree. Returns a dict with the kind,
    the anchor(s), both sides' values and |value - threshold| on each side.
    exp_o / exp_g: each side's exp (None = vd_expf; "divide" / "torch" = torch's,
    oracle/bbox.py scores_boxes) -- with the same heads on both sides this explains
    what the exp substitution alone changes."""
    io, xo, fo = frame_result(oloc, oconf, pri, h, w, exp_o)
    ig, xg, fg = frame_result(gloc, gconf, pri, h, w, exp_g)
    if np.array_equal(io, ig) and np.array_equal(xo, xg):
        return None
    so, bo = obbox.scores_boxes(oloc, oconf, pri, exp_o)
    sg, bg = obbox.scores_boxes(gloc, gconf, pri, exp_g)
    co, cg = set(np.nonzero(so >= F32(0.5))[0].tolist()), set(np.nonzero(sg >= F32(0.5))[0].tolist())
    flips = sorted(co ^ cg)
    if flips:
        worst = max(flips, key=lambda k: min(abs(float(so[k]) - 0.5), abs(float(sg[k]) - 0.5)))
        return {"kind": "score", "anchor": int(worst), "n": len(flips), "oracle": float(so[worst]),
                "gpu": float(sg[worst]), "threshold": 0.5,
                "dist": max(abs(float(so[k]) - 0.5) for k in flips),
                "dist_gpu": max(abs(float(sg[k]) - 0.5) for k in flips),
                "delta": max(abs(float(so[k]) - float(sg[k])) for k in flips)}
    oo, byo = nms_log(bo, so)
    og, byg = nms_log(bg, sg)
    if not np.array_equal(oo, og):
        p = int(np.nonzero(oo != og)[0][0])
        a, b = int(oo[p]), int(og[p])
        return {"kind": "order", "anchor": a, "other": b, "oracle": float(so[a] - so[b]),
                "gpu": float(sg[a] - sg[b]), "threshold": 0.0,
                "dist": abs(float(so[a] - so[b])), "dist_gpu": abs(float(sg[a] - sg[b])),
                "delta": abs(float(so[a] - so[b]) - float(sg[a] - sg[b]))}
    for c in oo:
        c = int(c)
        if byo[c] != byg[c]:
            k = byo[c] if byo[c] >= 0 else byg[c]
            vo, vg = _iou(bo, k, c), _iou(bg, k, c)
            return {"kind": "iou", "anchor": c, "other": int(k), "oracle": vo, "gpu": vg, "threshold": 0.4,
                    "dist": abs(vo - 0.4), "dist_gpu": abs(vg - 0.4), "delta": abs(vo - vg)}
    d = np.argwhere(xo != xg)
    r, q = (int(d[0][0]), int(d[0][1])) if len(d) else (0, 0)
    vo, vg = float(fo[r, q]), float(fg[r, q])
    # the integer the two floats straddle: int() truncates toward 0, so it is the
    # larger-magnitude of the two truncations
    t = float(xo[r, q] if abs(xo[r, q]) > abs(xg[r, q]) else xg[r, q])
    return {"kind": "trunc", "anchor": int(io[r]), "coord": q, "oracle": vo, "gpu": vg, "threshold": t,
            "dist": abs(vo - t), "dist_gpu": abs(vg - t), "delta": abs(vo - vg)}


def margin_stats(oloc, oconf, gloc, gconf, pri):
    """Largest forward-rounding differences over one frame's candidates (score >= 0.45
    on either side): |Δscore| and |Δbox| in canvas units."""
    so, sg = obbox.softmax2(oconf)[:, 1], obbox.softmax2(gconf)[:, 1]
    m = (so >= 0.45) | (sg >= 0.45)
    if not m.any():
        return 0.0, 0.0
    bo, bg = obbox.decode(oloc[m], pri[m]), obbox.decode(gloc[m], pri[m])
    return float(np.abs(so[m] - sg[m]).max()), float(np.abs(bo - bg).max())
