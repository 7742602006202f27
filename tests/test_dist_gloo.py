"""N > 1 path on CPU: world_size 2 and 4 over gloo (127.0.0.1).

SURVEY.md §8(e)'s rule, on one burst: every rank splits the SAME burst with
the RSS split of librxgpu (rxg_rss_split: the multi-queue NIC the reference's
README assumes, README.md:13, in place of its single queue, netfamily.c:38-39),
classifies its own shard, and reduces its per-flow counts with the path's one
collective.  Checks: the per-shard verdicts, put back in burst order through
the split's permutation, equal the verdicts of the unsharded burst; the
all-reduced counts equal the unsharded histogram; every frame of a shard
hashes to that shard by the oracle's independent Toeplitz restatement.

On CPU each shard is classified by the oracle (the checker) and the counts
are reduced over gloo; the -m gpu variant runs each rank's shard through its
own librxgpu context (the HIP path).  The same split + classify + RCCL reduce
runs in tests/test_multigpu.py (one GPU, two contexts) and in bench.py
--gpus N (one rank per GPU)."""
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


def _burst(name):
    cfg = rxdist.gen_cfg(name, n_udp=256, n_tcp=255)
    pk, off, ln = R.gen_host(cfg, 0, N_FRAMES, 6)
    udp, tcb = R.gen_flows(cfg)
    return pk, off, ln, udp, tcb


def _frame_shard(pk, o, l, world):
    """independent shard rule: oracle Toeplitz over the frame's tuple"""
    b = pk[int(o) << 6:(int(o) << 6) + 48].tobytes()
    b = b[:int(l)] + b"\0" * (48 - min(int(l), 48))
    if b[12:14] != b"\x08\x00":
        return 0
    sip, dip = int.from_bytes(b[26:30], "little"), int.from_bytes(b[30:34], "little")
    l4 = b[23] in (6, 17)
    sp = int.from_bytes(b[34:36], "little") if l4 else 0
    dp = int.from_bytes(b[36:38], "little") if l4 else 0
    return O.rss_hash(sip, dip, sp, dp) % world


def _worker(rank, world, port, name, q, gpu=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        pk, off, ln, udp, tcb = _burst(name)
        first, perm = R.rss_split(pk, off, ln, 6, world)
        mine = perm[first[rank]:first[rank + 1]]
        bad = sum(_frame_shard(pk, off[i], ln[i], world) != rank for i in mine)
        if gpu:  # the HIP path: this rank's own context on the box's GPU
            with R.Context(0, max_pkts=N_FRAMES, max_bytes=N_FRAMES * 1536) as ctx:
                ctx.flows_sync(udp, tcb)
                v = ctx.classify(pk, np.ascontiguousarray(off[mine]),
                                 np.ascontiguousarray(ln[mine]), 6)
                cnt = ctx.flow_counts()
        else:
            v, cnt = O.Tables(udp, tcb).classify(pk, off[mine], ln[mine], 6, counts=True)
        t = torch.from_numpy(cnt.astype(np.int64))
        work = rxdist.allreduce_counts(t, world, async_op=True)
        work.wait()
        q.put((rank, bad, mine.copy(), v.tobytes(), t.numpy().copy()))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("name,world", [("cfg2", 2), ("cfg4", 2), ("cfg4", 4)])
def test_rank_split_parity_and_count_reduce(name, world):
    _split_run(name, world, gpu=False)


@pytest.mark.gpu
@pytest.mark.parametrize("name,world", [("cfg4", 2)])
def test_rank_split_parity_and_count_reduce_hip(name, world):
    """the same, each rank classifying its shard through its own librxgpu
    context on the GPU (the ranks share the box's one GPU; gloo reduces)"""
    import torch as _t
    if not _t.cuda.is_available():
        pytest.fail("GPU tests need a GPU (no fallback path exists)")
    _split_run(name, world, gpu=True)


def _split_run(name, world, gpu):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, name, q, gpu))
             for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    pk, off, ln, udp, tcb = _burst(name)
    want, wcnt = O.Tables(udp, tcb).classify(pk, off, ln, 6, counts=True)
    got = np.zeros(N_FRAMES, R.VERDICT_DTYPE)
    seen = np.zeros(N_FRAMES, np.int64)
    for rank, bad, mine, vb, cnt in out:
        assert bad == 0, f"rank {rank}: {bad} frames outside its RSS shard"
        assert np.all(np.diff(mine.astype(np.int64)) > 0), "shard not in burst order"
        got[mine] = np.frombuffer(vb, R.VERDICT_DTYPE)
        seen[mine] += 1
        assert np.array_equal(cnt, wcnt.astype(np.int64)), rank
    assert np.all(seen == 1), "the shards do not partition the burst"
    assert got.tobytes() == want.tobytes()
    sizes = sorted(len(o[2]) for o in out)
    assert sizes[0] > 0.6 * N_FRAMES / world, sizes  # every shard carries traffic


@pytest.mark.parametrize("nsh", [1, 2, 3, 8, 64])
def test_host_split_matches_oracle_shards(nsh):
    """rxg_rss_split on mixed traffic (ARP/ICMP, runts, truncated captures):
    each shard is exactly the frames the oracle's Toeplitz puts there, in
    burst order, and first[] delimits them"""
    cfg = rxdist.gen_cfg("cfg4", n_udp=300, n_tcp=300, other_per10k=800)
    pk, off, ln = R.gen_host(cfg, 7, 2000, 6)
    rng = np.random.default_rng(nsh)
    ln = ln.copy()
    cut = rng.random(2000) < 0.05
    ln[cut] = rng.integers(0, 40, cut.sum())  # captures that end inside the tuple
    first, perm = R.rss_split(pk, off, ln, 6, nsh)
    assert first[0] == 0 and first[nsh] == 2000
    want = np.array([_frame_shard(pk, off[i], ln[i], nsh) for i in range(2000)])
    for s in range(nsh):
        sl = perm[first[s]:first[s + 1]]
        assert np.array_equal(sl, np.nonzero(want == s)[0]), s


def test_split_rejects_bad_shard_counts():
    pk, off, ln = R.gen_host(rxdist.gen_cfg("cfg2"), 0, 10, 6)
    for nsh in (0, R.MAX_SHARDS + 1):
        with pytest.raises(R.RxgError):
            R.rss_split(pk, off, ln, 6, nsh)
