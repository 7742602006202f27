"""Workload definitions (BASELINE.json configs) and the multi-GPU pieces:
RSS sharding of the synthetic traffic and the per-flow count reduction.

The rx path partitions naturally: every frame's verdict depends only on its
own bytes and the (replicated, read-only) flow table, so ranks classify their
RSS shard with no data-path collective.  The one exchange is the per-flow
packet count vector, summed over ranks with an all-reduce (RCCL over xGMI on
the GPU box, gloo in the CPU tests).  SURVEY.md §8(e).
"""
from __future__ import annotations

import rxgpu as R

# per-GPU workloads (weak scaling: the per-GPU work is fixed as N grows)
WORKLOADS = {
    # BASELINE configs[1]: 64 B UDP/IPv4, 1024 flows (sockets bound to :20000-21023)
    "cfg2": dict(desc="64B UDP/IPv4, 1024 flows, 16M frames/GPU", n=16 << 20, unit_log2=6,
                 len_hint=64,
                 gen=dict(frame_len=64, slot_bytes=64, proto_mode=0, n_udp=1024, n_tcp=0)),
    # BASELINE configs[2]: 1500 B TCP, 4096 established tcbs -> :9999 (+ the listener)
    "cfg3": dict(desc="1500B TCP/IPv4, 4096 tcbs + listener, 4M frames/GPU", n=4 << 20,
                 unit_log2=6, len_hint=1500,
                 gen=dict(frame_len=1500, slot_bytes=1536, proto_mode=1, n_udp=0, n_tcp=4096)),
    # BASELINE configs[3]: IMIX 64/576/1500 at 7:4:1, TCP/UDP 50/50, 64K flows; frames
    # packed at 64-B alignment (the layout the host staging path produces)
    "cfg4": dict(desc="IMIX 64/576/1500 (7:4:1), TCP+UDP, 65536 flows, 16M frames/GPU, packed",
                 n=16 << 20, unit_log2=6, len_hint=354,
                 gen=dict(size_mode=1, slot_bytes=1536, proto_mode=2, n_udp=32768, n_tcp=32767,
                          packed=1)),
    # BASELINE configs[4]: 10M x 9000 B TCP over 8 GPUs (1.25M/GPU), 1M tcbs
    "cfg5": dict(desc="9000B TCP jumbo, 1M tcbs, 1.25M frames/GPU (10M over 8 GPUs)",
                 n=1250000, unit_log2=6, len_hint=9000,
                 gen=dict(frame_len=9000, slot_bytes=9024, proto_mode=1, n_udp=0,
                          n_tcp=1048575)),
}


def gen_cfg(name: str, rank: int = 0, world: int = 1, **over) -> R.GenCfg:
    w = WORKLOADS[name]
    kw = dict(w["gen"])
    kw.update(seed=0x5EED0001 + int(name[3:]), shard=rank, n_shards=world)
    kw.update(over)
    return R.make_gen_cfg(**kw)


def allreduce_counts(counts, world: int, async_op: bool = False):
    """The single collective of the rx path: per-flow count vector sum.
    async_op=True returns the collective's work handle (overlap with the next
    burst's kernel; .wait() before reusing the buffer), else None."""
    if world > 1:
        import torch.distributed as dist
        return dist.all_reduce(counts, op=dist.ReduceOp.SUM, async_op=async_op)
    return None
