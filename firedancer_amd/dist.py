"""Multi-GPU plumbing for the data-parallel verify path (one process per GPU).

Signatures are independent, so the data path has NO collective: every rank
verifies its own contiguous shard on its own GPU.  torch.distributed is used
only for the benchmark's barrier / MAX-over-ranks timing and for an optional
host-side gather of per-shard result codes (the "host gather" of SURVEY.md
§8(e)); both work with the gloo backend (CPU tests) and nccl (= RCCL)."""
import torch
import torch.distributed as dist

from .shard import shard_range


def aggregate_throughput(local_items, local_seconds, device=None):
    """-> (total items over ranks, max seconds over ranks)."""
    t = torch.tensor([float(local_items), float(local_seconds)], dtype=torch.float64, device=device)
    if dist.is_initialized() and dist.get_world_size() > 1:
        items = t[:1].clone(); secs = t[1:].clone()
        dist.all_reduce(items, op=dist.ReduceOp.SUM)
        dist.all_reduce(secs, op=dist.ReduceOp.MAX)
        return float(items.item()), float(secs.item())
    return float(t[0].item()), float(t[1].item())


def gather_codes(local_codes, n, device=None):
    """Concatenate every rank's int8 code shard (rank order == shard order) -> full length-n array."""
    world = dist.get_world_size() if dist.is_initialized() else 1
    if world == 1:
        return local_codes
    maxlen = max(b - a for a, b in (shard_range(n, i, world) for i in range(world)))
    buf = torch.zeros(maxlen, dtype=torch.int8, device=device)
    buf[:len(local_codes)] = torch.as_tensor(local_codes, dtype=torch.int8, device=device)
    outs = [torch.zeros(maxlen, dtype=torch.int8, device=device) for _ in range(world)]
    dist.all_gather(outs, buf)
    parts = []
    for i in range(world):
        a, b = shard_range(n, i, world)
        parts.append(outs[i][:b - a].cpu())
    return torch.cat(parts).numpy()
