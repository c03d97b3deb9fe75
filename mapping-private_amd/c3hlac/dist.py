"""Frame sharding over ranks and the detection gather.

Frames are independent, so rank r of W processes frames r, r+W, r+2W, ... with no
data-path collective.  After a batch, every rank's M x rank detection records (c3h_det:
double score + 4 int32, viewed as 3 int64 words) are gathered with a single all_gather
(RCCL on the GPU, gloo in the CPU tests) and re-ordered by frame index.
"""
import torch


def frame_shard(n_frames, rank, world):
    """Frame indices owned by `rank` (round-robin)."""
    return list(range(rank, n_frames, world))


def gather_records(local, n_frames, rank, world, dist):
    """local: (len(frame_shard(...)), K) int64 tensor of this rank's records, in shard
    order.  Returns the (n_frames, K) tensor of all frames in frame order (every rank)."""
    per = (n_frames + world - 1) // world
    K = local.shape[1]
    buf = torch.zeros((per, K), dtype=local.dtype, device=local.device)
    buf[: local.shape[0]] = local
    parts = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(parts, buf)
    out = torch.empty((n_frames, K), dtype=local.dtype, device=local.device)
    for r in range(world):
        idx = frame_shard(n_frames, r, world)
        out[idx] = parts[r][: len(idx)]
    return out
