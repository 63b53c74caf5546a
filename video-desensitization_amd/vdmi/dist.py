"""Multi-GPU frame sharding.

The reference's only multi-GPU mechanism is nn.DataParallel inside one process
(detect_face/face.py:55-56): every forward re-broadcasts ~109 MB of fp32 weights,
scatters the input and gathers (loc, conf, landm) to cuda:0. Here frames are
independent units, so the MI355X design is one process per GPU over
torch.distributed (backend "nccl" = RCCL on ROCm):

* rank r owns the contiguous frame range [r*N/G, (r+1)*N/G) of a video, in
  batches of B; weights are uploaded once per rank; pixels never leave their GPU;
* the only exchange is an all-gather of fixed-size per-frame box records
  ``[count, x1, y1, x2, y2, ...]`` (int32, 1 + 4*cap words) over xGMI, so every
  rank (or the writer) sees the whole batch's detections. At cap=64 that is
  ~1 KB per frame, tens of KB per rank per step: latency-bound, far below one
  xGMI link's ~153 GB/s, so a single ring all-gather is the right collective.
"""
import numpy as np


def shard_range(n_frames, world, rank):
    """Contiguous [begin, end) frame range of `rank` (sizes differ by at most 1)."""
    base, rem = divmod(n_frames, world)
    begin = rank * base + min(rank, rem)
    return begin, begin + base + (1 if rank < rem else 0)


def pack_records(count, xyxy, cap):
    """int32 [n, 1 + 4*cap]: per frame the kept-box count then its int boxes
    (first `cap` of them; count may exceed cap, as vd_boxes reports it)."""
    import torch
    n = count.shape[0]
    rec = torch.zeros((n, 1 + 4 * cap), dtype=torch.int32, device=count.device)
    rec[:, 0] = count
    rec[:, 1:] = xyxy[:, :cap].reshape(n, 4 * cap)
    return rec


def unpack_records(rec):
    """-> list (per frame) of int (x1, y1, x2, y2) tuples."""
    rec = rec.cpu().numpy() if hasattr(rec, "cpu") else np.asarray(rec)
    cap = (rec.shape[1] - 1) // 4
    out = []
    for r in rec:
        k = min(int(r[0]), cap)
        out.append([tuple(int(v) for v in r[1 + 4 * i:5 + 4 * i]) for i in range(k)])
    return out


def all_gather_records(rec, group=None):
    """all_gather_into_tensor of equal-shaped per-rank record blocks -> [world*n, W]."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    out = torch.empty((world * rec.shape[0], rec.shape[1]), dtype=rec.dtype, device=rec.device)
    if rec.device.type == "cuda":
        dist.all_gather_into_tensor(out, rec.contiguous(), group=group)
    else:   # gloo has no all_gather_into_tensor on every build: list form
        parts = [torch.empty_like(rec) for _ in range(world)]
        dist.all_gather(parts, rec.contiguous(), group=group)
        out = torch.cat(parts, 0)
    return out
