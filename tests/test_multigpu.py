"""Multi-GPU path on one GPU, through the C ABI: RSS split on the device,
shard gather, two contexts classifying the two shards of ONE burst, the RCCL
count all-reduce (a one-rank communicator: the only group one GPU can form),
and contexts used from several threads / streams at once.

SURVEY.md §8(e): per-shard verdicts re-ordered by packet index equal the
one-GPU verdicts (and the oracle's); the per-shard counts summed equal the
one-GPU histogram.  The N-GPU run of the same code is bench.py --gpus N."""
import threading

import numpy as np
import pytest

import oracle_bind as O
import rxdist
import rxgpu as R

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_dev():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a GPU (no fallback path exists)")
    return torch, torch.device("cuda", 0)


def _to_dev(torch, dev, pk, off, ln):
    d_pk = torch.from_numpy(np.concatenate([pk, np.zeros(64, np.uint8)])).to(dev)
    d_off = torch.from_numpy(off.view(np.int32)).to(dev)
    d_ln = torch.from_numpy(ln.view(np.int16)).to(dev)
    return d_pk, d_off, d_ln


def _mixed_burst(n, nu=3000, nt=3000, first=17):
    cfg = rxdist.gen_cfg("cfg4", n_udp=nu, n_tcp=nt, other_per10k=300)
    pk, off, ln = R.gen_host(cfg, first, n, 6)
    udp, tcb = R.gen_flows(cfg)
    return pk, off, ln, udp, tcb


@pytest.mark.parametrize("nsh", [2, 3, 8])
def test_device_split_equals_host_split(torch_dev, nsh):
    torch, dev = torch_dev
    pk, off, ln, _, _ = _mixed_burst(50000)
    ln = ln.copy()
    ln[::97] = np.arange(len(ln[::97])) % 40  # captures ending inside the tuple
    hf, hp = R.rss_split(pk, off, ln, 6, nsh)
    d_pk, d_off, d_ln = _to_dev(torch, dev, pk, off, ln)
    d_first = torch.zeros(nsh + 1, dtype=torch.int32, device=dev)
    d_perm = torch.zeros(len(off), dtype=torch.int32, device=dev)
    with R.Context(0) as ctx:
        ctx.rss_split_dev(d_pk, d_off, d_ln, len(off), 6, nsh, d_first, d_perm,
                          stream=torch.cuda.current_stream(dev).cuda_stream)
        torch.cuda.synchronize(dev)
    assert np.array_equal(d_first.cpu().numpy().view(np.uint32), hf)
    assert np.array_equal(d_perm.cpu().numpy().view(np.uint32), hp)


def test_two_contexts_classify_the_shards_of_one_burst(torch_dev):
    torch, dev = torch_dev
    n, nsh = 60000, 2
    pk, off, ln, udp, tcb = _mixed_burst(n)
    want, wcnt = O.Tables(udp, tcb).classify(pk, off, ln, 6, counts=True)
    d_pk, d_off, d_ln = _to_dev(torch, dev, pk, off, ln)
    ctxs = [R.Context(0) for _ in range(nsh)]
    streams = [torch.cuda.Stream(dev) for _ in range(nsh)]
    try:
        for c in ctxs:
            c.flows_sync(udp, tcb)
        d_first = torch.zeros(nsh + 1, dtype=torch.int32, device=dev)
        d_perm = torch.zeros(n, dtype=torch.int32, device=dev)
        ctxs[0].rss_split_dev(d_pk, d_off, d_ln, n, 6, nsh, d_first, d_perm,
                              stream=torch.cuda.current_stream(dev).cuda_stream)
        torch.cuda.synchronize(dev)
        first = d_first.cpu().numpy().view(np.uint32)
        shards = []
        for r in range(nsh):  # the DMA of each queue's frames into its own burst
            cnt = int(first[r + 1] - first[r])
            idx = d_perm[int(first[r]):int(first[r + 1])]
            cap = cnt * 1536 + 64
            dst = torch.zeros(cap, dtype=torch.uint8, device=dev)
            doff = torch.zeros(cnt, dtype=torch.int32, device=dev)
            dlen = torch.zeros(cnt, dtype=torch.int16, device=dev)
            span = ctxs[r].gather_dev(d_pk, d_off, d_ln, 6, idx, cnt, dst, cap, doff, dlen,
                                      stream=torch.cuda.current_stream(dev).cuda_stream)
            assert 0 < span <= cap
            shards.append((idx, cnt, dst, doff, dlen))
        # gathered frames are byte-identical to the burst's
        h = shards[0]
        hidx = h[0].cpu().numpy().view(np.uint32)
        hdst, hoff, hlen = h[2].cpu().numpy(), h[3].cpu().numpy().view(np.uint32), \
            h[4].cpu().numpy().view(np.uint16)
        for k in range(0, h[1], 997):
            i = int(hidx[k])
            a, b = int(off[i]) << 6, int(hoff[k]) << 6
            assert hlen[k] == ln[i]
            assert hdst[b:b + int(ln[i])].tobytes() == pk[a:a + int(ln[i])].tobytes()
        # both contexts classify concurrently, each on its own stream
        outs, cnts = [], []
        for r, (idx, cnt, dst, doff, dlen) in enumerate(shards):
            o = torch.empty(cnt * 16, dtype=torch.uint8, device=dev)
            c = torch.zeros(ctxs[r].num_flows, dtype=torch.int64, device=dev)
            ctxs[r].classify_dev(dst, doff, dlen, cnt, 6, 354, o, c,
                                 stream=streams[r].cuda_stream)
            outs.append(o)
            cnts.append(c)
        torch.cuda.synchronize(dev)
        got = np.zeros(n, R.VERDICT_DTYPE)
        total = np.zeros(len(wcnt), np.uint64)
        for (idx, cnt, *_), o, c in zip(shards, outs, cnts):
            got[idx.cpu().numpy().view(np.uint32)] = o.cpu().numpy().view(R.VERDICT_DTYPE)
            total += c.cpu().numpy().view(np.uint64)
        assert got.tobytes() == want.tobytes()
        assert np.array_equal(total, wcnt)
    finally:
        for c in ctxs:
            c.close()


def test_rccl_group_one_rank(torch_dev):
    """rxg_group over one GPU: the communicator reports one rank
    (rxg_group_size, which the N-GPU bench line carries as rccl_nranks), and
    the all-reduce is the identity (sum over one rank), through the same
    ncclAllReduce call the N-GPU bench makes"""
    torch, dev = torch_dev
    g = R.Group(0, 1, 0, R.group_id())
    try:
        assert g.size() == (1, 0)  # rxg_group_size: what the communicator reports
        x = torch.arange(5000, dtype=torch.int64, device=dev) * 3
        y = x.clone()
        g.allreduce(y, 5000, stream=torch.cuda.current_stream(dev).cuda_stream)
        torch.cuda.synchronize(dev)
        assert torch.equal(x, y)
        pk, off, ln, udp, tcb = _mixed_burst(3000)
        with R.Context(0, max_pkts=4096, max_bytes=1 << 23) as ctx:
            ctx.flows_sync(udp, tcb)
            ctx.classify(pk, off, ln, 6)
            ctx.counts_allreduce(g)
            _, wcnt = O.Tables(udp, tcb).classify(pk, off, ln, 6, counts=True)
            assert np.array_equal(ctx.flow_counts(), wcnt)
    finally:
        g.close()


def test_contexts_on_concurrent_threads(torch_dev):
    """one rxg_ctx per rx thread (rxgpu.h): two threads, flow sets of
    different sizes (LDS histogram vs slab counts, different launch shapes),
    bursts in flight at the same time; every verdict and count bit-exact"""
    torch, dev = torch_dev
    jobs = [_mixed_burst(20000, 512, 511, first=5), _mixed_burst(20000, 6000, 6000, first=9)]
    results = [None, None]
    errors = []

    def run(k):
        try:
            pk, off, ln, udp, tcb = jobs[k]
            torch.cuda.set_device(dev)
            s = torch.cuda.Stream(dev)
            with R.Context(0) as ctx:
                ctx.flows_sync(udp, tcb)
                d_pk, d_off, d_ln = _to_dev(torch, dev, pk, off, ln)
                c = torch.zeros(ctx.num_flows, dtype=torch.int64, device=dev)
                o = torch.empty(len(off) * 16, dtype=torch.uint8, device=dev)
                for it in range(12):
                    ctx.classify_dev(d_pk, d_off, d_ln, len(off), 6, (64, 354, 1500)[it % 3], o, c,
                                     stream=s.cuda_stream)
                s.synchronize()
                results[k] = (o.cpu().numpy().view(R.VERDICT_DTYPE).copy(),
                              c.cpu().numpy().view(np.uint64).copy())
        except Exception as e:  # surfaced below
            errors.append(e)

    ts = [threading.Thread(target=run, args=(k,)) for k in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    assert not errors, errors
    for k, (pk, off, ln, udp, tcb) in enumerate(jobs):
        want, wcnt = O.Tables(udp, tcb).classify(pk, off, ln, 6, counts=True)
        assert results[k][0].tobytes() == want.tobytes(), k
        assert np.array_equal(results[k][1], 12 * wcnt), k


def test_one_context_two_streams_share_workspace(torch_dev):
    """bursts of one context on two streams, back to back, on the slab count
    path (its workspace is per context): the second waits for the first"""
    torch, dev = torch_dev
    pk, off, ln, udp, tcb = _mixed_burst(40000, 6000, 6000)
    want, wcnt = O.Tables(udp, tcb).classify(pk, off, ln, 6, counts=True)
    d_pk, d_off, d_ln = _to_dev(torch, dev, pk, off, ln)
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    with R.Context(0) as ctx:
        ctx.flows_sync(udp, tcb)
        c1 = torch.zeros(ctx.num_flows, dtype=torch.int64, device=dev)
        c2 = torch.zeros(ctx.num_flows, dtype=torch.int64, device=dev)
        o1 = torch.empty(len(off) * 16, dtype=torch.uint8, device=dev)
        o2 = torch.empty(len(off) * 16, dtype=torch.uint8, device=dev)
        for _ in range(4):
            ctx.classify_dev(d_pk, d_off, d_ln, len(off), 6, 354, o1, c1, stream=s1.cuda_stream)
            ctx.classify_dev(d_pk, d_off, d_ln, len(off), 6, 354, o2, c2, stream=s2.cuda_stream)
        torch.cuda.synchronize(dev)
    for o, c in ((o1, c1), (o2, c2)):
        assert o.cpu().numpy().view(R.VERDICT_DTYPE).tobytes() == want.tobytes()
        assert np.array_equal(c.cpu().numpy().view(np.uint64), 4 * wcnt)


@pytest.mark.parametrize("nu,nt,n", [(6000, 6000, 40000), (40000, 30000, 12000), (300, 300, 40000)])
def test_counts_on_a_second_stream(torch_dev, nu, nt, n):
    """rxg_classify_dev_cs: verdicts on the classify stream, the slab count on a
    count stream, overlapping the next burst's classify (two index buffers in
    the context).  Two different bursts alternate, a plain rxg_classify_dev
    burst and a burst of another size (the workspace regions move) are mixed
    in: every verdict is bit-exact and the counts add up to the histograms.
    With few flows the classify kernel counts itself (no slab passes) and the
    count stream is still ordered after it"""
    torch, dev = torch_dev
    cfg = rxdist.gen_cfg("cfg4", n_udp=nu, n_tcp=nt, other_per10k=300)
    udp, tcb = R.gen_flows(cfg)
    tb = O.Tables(udp, tcb)
    bursts = []
    for first, m in ((17, n), (5 * n, n), (9 * n, n // 2 + 3)):
        pk, off, ln = R.gen_host(cfg, first, m, 6)
        want, wcnt = tb.classify(pk, off, ln, 6, counts=True)
        bursts.append((_to_dev(torch, dev, pk, off, ln), m, want, wcnt))
    s, cs = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    order = [0, 1, 0, 1, 1, 2, 0, 2, 1, 0]  # burst index per step
    plain = {3, 7}                           # these steps use rxg_classify_dev on s
    with R.Context(0) as ctx:
        ctx.flows_sync(udp, tcb)
        cnt = torch.zeros(ctx.num_flows, dtype=torch.int64, device=dev)
        outs = []
        for k, b in enumerate(order):
            (d_pk, d_off, d_ln), m, _, _ = bursts[b]
            o = torch.empty(m * 16, dtype=torch.uint8, device=dev)
            if k in plain:
                s.wait_stream(cs)  # the caller orders its own count target
                ctx.classify_dev(d_pk, d_off, d_ln, m, 6, 354, o, cnt, stream=s.cuda_stream)
                cs.wait_stream(s)
            else:
                ctx.classify_dev(d_pk, d_off, d_ln, m, 6, 354, o, cnt, stream=s.cuda_stream,
                                 count_stream=cs.cuda_stream)
            outs.append(o)
        torch.cuda.synchronize(dev)
    want_cnt = sum(bursts[b][3].astype(np.uint64) for b in order)
    for k, b in enumerate(order):
        got = outs[k].cpu().numpy().view(R.VERDICT_DTYPE)
        assert got.tobytes() == bursts[b][2].tobytes(), k
    assert np.array_equal(cnt.cpu().numpy().view(np.uint64), want_cnt)
