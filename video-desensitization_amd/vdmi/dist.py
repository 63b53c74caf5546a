"""Multi-GPU frame sharding.

The reference's only multi-GPU mechanism is nn.DataParallel inside one process
(detect_face/face.py:55-56): every forward re-broadcasts ~109 MB of fp32 weights,
scatters the input and gathers (loc, conf, landm) to cuda:0. Here frames are
independent units, so the MI355X design is one process per GPU over
torch.distributed (backend "nccl" = RCCL on ROCm):

* rank r owns the contiguous frame range [r*N/G, (r+1)*N/G) of a video, in
  batches of B; weights are uploaded once per rank; pixels never leave their GPU;
* the only exchange is an all-gather of fixed-size per-frame box records
  ``[frame, count, 64 x (x1, y1, x2, y2), 64 x score, 64 x anchor]`` (int32,
  2 + 6*cap words) over xGMI, so every rank (or the writer) sees the whole
  batch's detections. At cap=64 that is ~1.5 KB per frame, ~100 KB per rank per
  step: latency-bound, far below one xGMI link's ~153 GB/s, so a single ring
  all-gather is the right collective. Uneven shards pad to the largest with
  frame = -1 rows (all_gather_into_tensor needs equal blocks).
"""
import numpy as np


def shard_range(n_frames, world, rank):
    """Contiguous [begin, end) frame range of `rank` (sizes differ by at most 1)."""
    base, rem = divmod(n_frames, world)
    begin = rank * base + min(rank, rem)
    return begin, begin + base + (1 if rank < rem else 0)


REC_HDR = 2   # words before the boxes: frame index, count


def rec_width(cap):
    """int32 words per frame record: frame, count, cap boxes, cap scores, cap anchors."""
    return REC_HDR + 6 * cap


def pack_records(count, xyxy, cap, score=None, anchor=None, frame=None):
    """int32 [n, 2 + 6*cap] per-frame records: global frame index,
    kept-box count (complete, may exceed cap), then the first `cap` int boxes,
    their f32 scores (bit pattern) and anchor indices. Padding rows use frame -1."""
    import torch
    n = count.shape[0]
    dev = count.device
    rec = torch.zeros((n, rec_width(cap)), dtype=torch.int32, device=dev)
    rec[:, 0] = frame if frame is not None else torch.arange(n, dtype=torch.int32, device=dev)
    rec[:, 1] = count
    k = min(cap, xyxy.shape[1])
    rec[:, 2:2 + 4 * k] = xyxy[:, :k].reshape(n, 4 * k)
    if score is not None:
        rec[:, 2 + 4 * cap:2 + 4 * cap + k] = score[:, :k].contiguous().view(torch.int32)
    if anchor is not None:
        rec[:, 2 + 5 * cap:2 + 5 * cap + k] = anchor[:, :k]
    return rec


def unpack_records(rec):
    """-> {frame: (boxes [(x1, y1, x2, y2)], scores [float], anchors [int], count)} for
    every non-padding record; boxes/scores/anchors hold min(count, cap) entries."""
    rec = rec.cpu().numpy() if hasattr(rec, "cpu") else np.asarray(rec)
    rec = np.ascontiguousarray(rec, np.int32)
    cap = (rec.shape[1] - REC_HDR) // 6
    out = {}
    for r in rec:
        f = int(r[0])
        if f < 0:
            continue
        k = min(int(r[1]), cap)
        boxes = [tuple(int(v) for v in r[2 + 4 * i:6 + 4 * i]) for i in range(k)]
        scores = r[2 + 4 * cap:2 + 4 * cap + k].view(np.float32).tolist()
        anchors = [int(v) for v in r[2 + 5 * cap:2 + 5 * cap + k]]
        out[f] = (boxes, scores, anchors, int(r[1]))
    return dict(sorted(out.items()))


def all_gather_records(rec, group=None):
    """all_gather_into_tensor of equal-shaped per-rank record blocks -> [world*n, W]."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    if rec.device.type == "cuda" and dist.get_backend(group) == "gloo":
        # gloo (CPU tests, bench --backend gloo): gather through host memory
        return all_gather_records(rec.cpu(), group).to(rec.device)
    out = torch.empty((world * rec.shape[0], rec.shape[1]), dtype=rec.dtype, device=rec.device)
    if rec.device.type == "cuda":
        dist.all_gather_into_tensor(out, rec.contiguous(), group=group)
    else:   # gloo has no all_gather_into_tensor on every build: list form
        parts = [torch.empty_like(rec) for _ in range(world)]
        dist.all_gather(parts, rec.contiguous(), group=group)
        out = torch.cat(parts, 0)
    return out
