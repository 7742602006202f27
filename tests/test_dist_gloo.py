"""N > 1 path on CPU: world_size 2 over gloo (127.0.0.1).

Each rank generates its RSS shard of a workload (the same pktgen the GPU
bench uses), computes its per-flow counts (here with the oracle: no GPU in
this container), and reduces them with rxdist.allreduce_counts, the single
collective of the rx path.  Checks: every rank's frames hash to that rank,
and the reduced counts equal the sum of the per-shard histograms computed
independently in one process."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle_bind as O
import rxdist
import rxgpu as R

N_FRAMES = 3000


def _shard(name, rank, world):
    cfg = rxdist.gen_cfg(name, rank, world, n_udp=256, n_tcp=255)
    pk, off, ln = R.gen_host(cfg, 0, N_FRAMES, 6)
    udp, tcb = R.gen_flows(cfg)
    v, cnt = O.Tables(udp, tcb).classify(pk, off, ln, 6, counts=True)
    return cfg, pk, off, v, cnt


def _worker(rank, world, port, name, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cfg, pk, off, v, cnt = _shard(name, rank, world)
        # every IP frame of this rank carries a tuple whose RSS hash picks this rank
        bad = 0
        for k in range(N_FRAMES):
            b = pk[int(off[k]) << 6:(int(off[k]) << 6) + 64].tobytes()
            if b[12:14] != b"\x08\x00":
                continue
            sip, dip = int.from_bytes(b[26:30], "little"), int.from_bytes(b[30:34], "little")
            l4 = b[23] in (6, 17)
            sp = int.from_bytes(b[34:36], "little") if l4 else 0
            dp = int.from_bytes(b[36:38], "little") if l4 else 0
            bad += O.rss_hash(sip, dip, sp, dp) % world != rank
        t = torch.from_numpy(cnt.astype(np.int64))
        work = rxdist.allreduce_counts(t, world, async_op=True)
        work.wait()
        q.put((rank, bad, t.numpy().copy()))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("name", ["cfg2", "cfg4"])
def test_two_rank_shard_and_count_reduce(name):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, name, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # single-process reference: the per-shard histograms, summed
    want = sum(_shard(name, r, world)[4].astype(np.int64) for r in range(world))
    for rank, bad, got in out:
        assert bad == 0, f"rank {rank}: {bad} frames outside its RSS shard"
        assert np.array_equal(got, want), rank
    assert want.sum() > 0.9 * world * N_FRAMES
