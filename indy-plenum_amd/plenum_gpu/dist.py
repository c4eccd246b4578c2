"""Multi-GPU sharding for the verify path.

One process per GPU.  Signatures are independent, so a batch of n is split
into contiguous index ranges (rank r owns [n*r/W, n*(r+1)/W)), each rank
verifies its shard with no data-path communication, and the only collective
is an all-gather of the packed verdict bitmaps (RCCL over xGMI with the
"nccl" backend on ROCm; gloo on CPU for tests).  3PC tally batches shard by
batch, so every tally is rank-local and only the quorum bits are gathered.

Bitmap layout: 64-bit words, bit i%64 of word i//64 = verdict of local
signature i; every rank pads its shard to `words_per_rank` words so the
gather is one fixed-size all_gather_into_tensor.
"""
import numpy as np


def shard_range(n, rank, world):
    """[start, stop) of rank's contiguous shard."""
    return n * rank // world, n * (rank + 1) // world


def words_per_rank(n, world):
    """Bitmap words per rank (the largest shard, rounded up to 64 bits)."""
    return (max(shard_range(n, r, world)[1] - shard_range(n, r, world)[0] for r in range(world)) + 63) // 64


def pack_bits(verdict, words):
    """bool[m] -> int64[words] (little-endian bit order within each word)."""
    v = np.zeros(words * 64, dtype=np.uint8)
    v[:len(verdict)] = np.asarray(verdict, dtype=np.uint8)
    return np.packbits(v, bitorder='little').view(np.int64)


def unpack_gathered(gathered, n, world):
    """int64[world*words] gathered bitmaps -> bool[n] in global index order."""
    words = gathered.size // world
    bits = np.unpackbits(np.ascontiguousarray(gathered).view(np.uint8), bitorder='little').astype(bool)
    out = np.zeros(n, dtype=bool)
    for r in range(world):
        s, e = shard_range(n, r, world)
        out[s:e] = bits[r * words * 64: r * words * 64 + (e - s)]
    return out


def gather_verdicts(bitmap_tensor, n, world, group=None):
    """all_gather_into_tensor of each rank's bitmap -> bool[n] (global order)."""
    import torch
    import torch.distributed as dist
    out = torch.empty(world * bitmap_tensor.numel(), dtype=bitmap_tensor.dtype, device=bitmap_tensor.device)
    dist.all_gather_into_tensor(out, bitmap_tensor, group=group)
    return unpack_gathered(out.cpu().numpy(), n, world)


def verify_sharded(pk, sig, blob, off, rank, world, verify_fn, group=None, device=None):
    """Verify this rank's shard with `verify_fn(pk, sig, blob, off) -> bool[]`
    and all-gather every rank's verdicts.  Inputs are the full batch on host
    (each rank slices its own range); returns bool[n] on every rank."""
    import torch
    n = len(pk)
    s, e = shard_range(n, rank, world)
    o = np.asarray(off, np.uint64)
    local_off = o[s:e + 1] - o[s]
    local = verify_fn(pk[s:e], sig[s:e], np.asarray(blob)[int(o[s]):int(o[e])], local_off)
    words = words_per_rank(n, world)
    bm = torch.from_numpy(pack_bits(local, words).copy())
    if device is not None:
        bm = bm.to(device)
    return gather_verdicts(bm, n, world, group)


def gather_quorums(reached_tensor, group=None):
    """all_gather_into_tensor of each rank's per-batch quorum flags (uint8, one
    per 3PC batch; every rank holds the same number of batches) -> bool[world*nb]
    in global batch order (C3: batches shard by batch, the tally is rank-local)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    out = torch.empty(world * reached_tensor.numel(), dtype=reached_tensor.dtype, device=reached_tensor.device)
    dist.all_gather_into_tensor(out, reached_tensor.contiguous(), group=group)
    return out
