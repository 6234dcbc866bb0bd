"""Best-rollout selection across ranks.

Rollouts are sharded into contiguous id ranges, one range per GPU; nothing is
exchanged while the path runs. At the end every rank encodes its rollouts'
(COT, global id) as an order-preserving 64-bit key (same encoding as
hs_best_key_encode) and the job performs ONE all_reduce(MIN) of 8 bytes
(RCCL over xGMI on GPUs, gloo in the CPU tests).
"""
from __future__ import annotations

import torch

_FLIP = -(2 ** 63)  # xor with the sign bit maps uint64 order onto int64 order
KEY_MIN_STEP_LENGTH = 1e-3  # HS_KEY_MIN_STEP_LENGTH


def select_cot(work: torch.Tensor, step_length: torch.Tensor, total_mass, n_t: int, steps: int) -> torch.Tensor:
    """hs_best_key_cot on a shard: one cycle's COT for forward or backward walking,
    work * (n_t / steps) / (total_mass * |L|), NaN where |L| < 1e-3 (include/hslabs.h). The same
    expression in the same precision and order as the device's key_cot, so the keys agree
    bitwise (work's dtype: float64, or float32 for HS_PREC_F32 runs)."""
    dt = work.dtype
    L = step_length.to(dt)
    aL = L.abs()
    r = torch.tensor(n_t, dtype=dt) / torch.tensor(steps, dtype=dt)
    m = torch.as_tensor(total_mass, dtype=dt, device=work.device)
    c = work * r.to(work.device) / (m * aL)
    return torch.where(aL >= KEY_MIN_STEP_LENGTH, c, torch.full_like(c, float("nan")))


def best_key(cot: torch.Tensor, id0: int) -> torch.Tensor:
    """Min key over one shard of selection COTs (float64 or float32 [B], NaN sorts last).
    Returns int64 [1] (sign-flipped, so int64 MIN is the uint64 key's MIN)."""
    c = cot.to(torch.float32)
    bits = c.view(torch.int32).to(torch.int64) & 0xFFFFFFFF
    ordk = torch.where(bits >= 0x80000000, (~bits) & 0xFFFFFFFF, bits | 0x80000000)
    ordk = torch.where(torch.isnan(c), torch.full_like(ordk, 0xFFFFFFFF), ordk)
    ids = torch.arange(id0, id0 + c.numel(), device=c.device, dtype=torch.int64) & 0xFFFFFFFF
    key = (ordk << 32) | ids
    return (key ^ _FLIP).min().reshape(1)


def reduce_best(key: torch.Tensor, group=None) -> torch.Tensor:
    """all_reduce(MIN) of a sign-flipped 8-byte key through torch.distributed (the gloo CPU
    tests and the bench's untimed cross-check; the GPU path's collective is hs_comm_reduce_best,
    RCCL inside libhslabs)."""
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(key, op=dist.ReduceOp.MIN, group=group)
    return key


def decode(key: torch.Tensor):
    """-> (cot as float32, global rollout id) from a sign-flipped key."""
    import struct

    u = (int(key.item()) ^ _FLIP) & 0xFFFFFFFFFFFFFFFF
    ordk, rid = u >> 32, u & 0xFFFFFFFF
    if ordk == 0xFFFFFFFF:
        return float("nan"), rid
    bits = (ordk & 0x7FFFFFFF) if ordk & 0x80000000 else (~ordk & 0xFFFFFFFF)
    return struct.unpack("<f", struct.pack("<I", bits))[0], rid


def shard(n_total: int, world: int, rank: int):
    """Contiguous rollout range of one rank: (id0, count)."""
    base, rem = divmod(n_total, world)
    count = base + (1 if rank < rem else 0)
    id0 = rank * base + min(rank, rem)
    return id0, count
