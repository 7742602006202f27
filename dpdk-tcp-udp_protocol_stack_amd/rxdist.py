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
    # BASELINE configs[0]: the reference's own CPU case — 100K x 64 B UDP from a pcap,
    # one flow: the echo client 10.0.0.1:5555 -> the echo socket 192.168.100.77:8889
    # (udp_server_entry, netfamily.c:227-229), every frame delivered (udp.c:4-57)
    "cfg1": dict(desc="64B UDP/IPv4 from pcap, 1 flow (10.0.0.1:5555 -> 192.168.100.77:8889), "
                      "100K frames", n=100000, unit_log2=6, len_hint=64,
                 gen=dict(frame_len=64, slot_bytes=64, proto_mode=0, n_udp=1, n_tcp=0,
                          udp_base_port=8889, src_ip=R.ip_raw("10.0.0.1"), src_port=5555,
                          bad_cksum_per10k=0, unknown_per10k=0, other_per10k=0)),
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
    """generator config of a workload; rank/world > 1 = the generator's own
    rejection-sampled RSS shard (frames of the shard only: the multi-GPU
    bench's default, build_shard mode "direct")."""
    w = WORKLOADS[name]
    kw = dict(w["gen"])
    kw.update(seed=0x5EED0001 + int(name[3:]), shard=rank, n_shards=world)
    kw.update(over)
    return R.make_gen_cfg(**kw)


def allreduce_counts(counts, world: int, async_op: bool = False):
    """The count reduction over torch.distributed (gloo in the CPU tests, where
    there is no RCCL); GPU ranks use rxgpu.Group (RCCL through the C ABI).
    async_op=True returns the work handle, else None."""
    if world > 1:
        import torch.distributed as dist
        return dist.all_reduce(counts, op=dist.ReduceOp.SUM, async_op=async_op)
    return None


def build_shard(ctx, name: str, rank: int, world: int, dev, stream, mode: str = "direct"):
    """This rank's share of a workload's burst, resident in HBM.

    world == 1: the burst itself (n frames).  world > 1:
      mode "direct" (the default): this rank's n frames generated straight
        into HBM by the generator's own RSS sharding (rxg_gen_cfg.shard /
        n_shards: only tuples whose rxg_rss_hash % world == rank) — the frames
        a multi-queue NIC would DMA into this GPU's queue, at one generation
        pass per rank;
      mode "split": the GLOBAL burst of world * n frames is generated chunk by
        chunk (n frames per chunk, frame i the same pure function of (cfg, i)
        on every rank), RSS-split on the device (rxg_rss_split_dev) and this
        rank's frames gathered into one packed burst (rxg_gather_dev), so the
        ranks' shards partition one burst whose first n frames carry golden
        digests (2 * world generation passes per rank).
    Returns (pk, off, ln, n_local, gidx, cfg): gidx = the global frame index
    of every local frame (int64, host; None when the frames are local indices
    of `cfg`'s stream), cfg = the generator config that regenerates them."""
    import numpy as np
    import torch
    w = WORKLOADS[name]
    cfg = gen_cfg(name)
    n, ul = w["n"], w["unit_log2"]
    sh = stream.cuda_stream
    if world == 1 or mode == "direct":
        if world > 1:
            cfg = gen_cfg(name, rank, world)
        pk = torch.empty(n * cfg.slot_bytes + 64, dtype=torch.uint8, device=dev)
        off = torch.empty(n, dtype=torch.int32, device=dev)
        ln = torch.empty(n, dtype=torch.int16, device=dev)
        R.gen_dev(cfg, 0, n, pk, off, ln, ul, stream=sh)
        torch.cuda.synchronize(dev)
        return pk, off, ln, n, None, cfg
    c_pk = torch.empty(n * cfg.slot_bytes + 64, dtype=torch.uint8, device=dev)
    c_off = torch.empty(n, dtype=torch.int32, device=dev)
    c_ln = torch.empty(n, dtype=torch.int16, device=dev)
    d_first = torch.zeros(world + 1, dtype=torch.int32, device=dev)
    d_perm = torch.empty(n, dtype=torch.int32, device=dev)

    def chunk(c):
        R.gen_dev(cfg, c * n, n, c_pk, c_off, c_ln, ul, stream=sh)
        ctx.rss_split_dev(c_pk, c_off, c_ln, n, ul, world, d_first, d_perm, stream=sh)
        torch.cuda.synchronize(dev)
        f = d_first.cpu().numpy().view(np.uint32)
        return int(f[rank]), int(f[rank + 1])

    # pass 1: this rank's frame count and packed size
    frames, units = 0, 0
    for c in range(world):
        a, b = chunk(c)
        idx = d_perm[a:b].long()
        lens = c_ln[idx].to(torch.int64).bitwise_and(0xFFFF)
        units += int(((lens + 63) // 64).clamp(min=1).sum().item())
        frames += b - a
    pk = torch.zeros(units * 64 + 64, dtype=torch.uint8, device=dev)
    off = torch.empty(max(frames, 1), dtype=torch.int32, device=dev)
    ln = torch.empty(max(frames, 1), dtype=torch.int16, device=dev)
    gidx = np.empty(frames, np.int64)
    # pass 2: regenerate, split, gather into place
    k0, pos = 0, 0
    for c in range(world):
        a, b = chunk(c)
        cnt = b - a
        if cnt == 0:
            continue
        used = ctx.gather_dev(c_pk, c_off, c_ln, ul, d_perm[a:b], cnt, pk.data_ptr() + pos,
                              pk.numel() - pos, off[k0:k0 + cnt], ln[k0:k0 + cnt], stream=sh)
        off[k0:k0 + cnt] += pos >> 6
        gidx[k0:k0 + cnt] = d_perm[a:b].cpu().numpy().view(np.uint32).astype(np.int64) + c * n
        k0 += cnt
        pos += used
    torch.cuda.synchronize(dev)
    del c_pk, c_off, c_ln, d_perm
    torch.cuda.empty_cache()
    return pk, off, ln, frames, gidx, cfg
