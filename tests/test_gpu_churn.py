"""Connection churn on the GPU, and the control plane's hygiene (-m gpu).

The reference creates a tcb on every SYN (tcp.c:50-52, LL_ADD) and frees it
on the last ACK and on close (tcp.c:321, common.c:620,660), while the rx loop
keeps classifying.  Here the context's tables follow with rxg_flows_add /
rxg_flows_remove (committed in stream order with the next burst: a few slot
writes, no rebuild, no device-wide synchronisation), and every burst's
verdicts are checked against the reference's lookups on the lists as they
stand at that burst: a model of the lists for every frame, and the oracle's
list scans (oracle/ref_cpu.c) for a sample, with its creation-order indices
mapped to the blocks' stable ids."""
import time

import numpy as np
import pytest

import frames as F
import oracle_bind as O
import rxdist
import rxgpu as R

pytestmark = pytest.mark.gpu
L = R.ip_raw("192.168.100.77")
P9999 = R.port_raw(9999)


@pytest.fixture(scope="module")
def torch_dev():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a GPU (no fallback path exists)")
    return torch, torch.device("cuda", 0)


class TcbLists:
    """the tcb list of the reference as stable ids: key = (sip, sport) (dip
    and dport are the local socket's), newest live block per key wins, else
    the listener (id 0: tcp_stream_search pass 2)"""

    def __init__(self, tcb):
        n = len(tcb)
        cap = n + 400000
        self.sip = np.zeros(cap, np.uint32)
        self.sport = np.zeros(cap, np.uint16)
        self.seq = np.zeros(cap, np.int64)
        self.alive = np.zeros(cap, bool)
        self.sip[:n], self.sport[:n] = tcb["sip"], tcb["sport"]
        self.seq[:n] = np.arange(n)
        self.alive[:n] = True
        self.next_seq = n
        self.keys = {}  # key -> [ids], creation order
        for i in range(1, n):
            self.keys.setdefault((int(tcb["sip"][i]) << 16) | int(tcb["sport"][i]), []).append(i)

    def add(self, fid, sip, sport):
        self.sip[fid], self.sport[fid] = sip, sport
        self.seq[fid] = self.next_seq
        self.next_seq += 1
        self.alive[fid] = True
        self.keys.setdefault((int(sip) << 16) | int(sport), []).append(fid)

    def remove(self, fid):
        self.alive[fid] = False
        k = (int(self.sip[fid]) << 16) | int(self.sport[fid])
        self.keys[k].remove(fid)
        if not self.keys[k]:
            del self.keys[k]

    def expect(self, sip, sport):
        ids = self.keys.get((int(sip) << 16) | int(sport))
        return ids[-1] if ids else 0

    def oracle(self):
        live = np.nonzero(self.alive)[0]
        order = live[np.argsort(self.seq[live], kind="stable")]
        t = np.zeros(len(order), R.TCB_DTYPE)
        t["sip"], t["dip"], t["sport"], t["dport"] = self.sip[order], L, self.sport[order], P9999
        t["status"] = R.TCP_STATUS_ESTABLISHED
        t["status"][order == 0] = R.TCP_STATUS_LISTEN
        return O.Tables(np.zeros(0, R.UDP_SOCK_DTYPE), t), order


def test_churn_1m_tcbs_bit_exact(torch_dev):
    """cfg5's 1M tcbs + listener; 100 bursts of 64K frames, before each one
    1000 tcbs removed and 1000 added (200 of them duplicates of live keys,
    which then win, and some keys removed this very burst re-added): every
    verdict's flow id / rc against the list model, a sample bit for bit
    against the oracle every 5th burst; the per-burst update cost is timed"""
    torch, dev = torch_dev
    cfg = rxdist.gen_cfg("cfg5")
    _, tcb = R.gen_flows(cfg)
    ctx = R.Context(0)
    ctx.flows_sync(None, tcb)
    m = TcbLists(tcb)
    rng = np.random.default_rng(2024)
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream
    nf = 65536
    d_pk = torch.empty(nf * 64 + 64, dtype=torch.uint8, device=dev)
    d_off = torch.arange(nf, dtype=torch.int32, device=dev)
    d_ln = torch.full((nf,), 64, dtype=torch.int16, device=dev)
    d_out = torch.empty(nf * 16, dtype=torch.uint8, device=dev)
    fresh = 0
    host_us, dev_us = [], []
    rebuilds0 = ctx.flows_rebuilds
    for b in range(100):
        live = np.nonzero(m.alive)[0]
        live = live[live != 0]
        gone = rng.choice(live, 1000, replace=False)
        dup_src = rng.choice(np.setdiff1d(live, gone), 200, replace=False)
        readd = gone[:50]
        add_sip = np.concatenate([(0x0A0000C8 + np.arange(fresh, fresh + 750)).astype(np.uint32)
                                  .byteswap(), m.sip[dup_src], m.sip[readd]])
        add_sport = np.concatenate([np.full(750, R.port_raw(4242), np.uint16), m.sport[dup_src],
                                    m.sport[readd]])
        fresh += 750
        t = np.zeros(1000, R.TCB_DTYPE)
        t["sip"], t["dip"], t["sport"], t["dport"] = add_sip, L, add_sport, P9999
        t["status"] = R.TCP_STATUS_ESTABLISHED
        gone_keys = (m.sip[gone].copy(), m.sport[gone].copy())
        h0 = time.perf_counter()
        ctx.flows_remove(None, gone)
        _, tid, _ = ctx.flows_add(None, t)
        host_us.append((time.perf_counter() - h0) * 1e6)
        for fid in gone:
            m.remove(int(fid))
        for k, fid in enumerate(tid):
            m.add(int(fid), add_sip[k], add_sport[k])
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        ctx.flows_commit(sh)
        e1.record(stream)
        # the burst: frames to the added keys, the removed keys, random live blocks
        live = np.nonzero(m.alive)[0]
        pick = rng.choice(live, nf - 2000)
        sip = np.concatenate([add_sip, gone_keys[0], m.sip[pick]])
        sport = np.concatenate([add_sport, gone_keys[1], m.sport[pick]])
        fr = F.tcp64_frames(sip, np.full(nf, L, np.uint32), sport, np.full(nf, P9999, np.uint16))
        d_pk[:nf * 64].copy_(torch.from_numpy(fr.reshape(-1)))
        ctx.classify_dev(d_pk, d_off, d_ln, nf, 6, 64, d_out, None, stream=sh)
        torch.cuda.synchronize(dev)
        dev_us.append(e0.elapsed_time(e1) * 1e3)
        v = d_out.cpu().numpy().view(R.VERDICT_DTYPE)
        want = np.array([m.expect(a, c) for a, c in zip(sip, sport)], np.uint32)
        bad = np.nonzero((v["flow_id"] != want) | (v["rc"] != 0) | (v["cls"] != R.CLS_TCP))[0]
        assert len(bad) == 0, (b, len(bad), [(int(i), v[i], want[i]) for i in bad[:3]])
        if b % 5 == 0:
            tb, order = m.oracle()
            smp = np.concatenate([np.arange(16), 1000 + np.arange(8), 2000 + rng.choice(nf - 2000, 8)])
            o = tb.classify(fr[smp].reshape(-1), np.arange(len(smp), dtype=np.uint32),
                            np.full(len(smp), 64, np.uint16), 6)
            o["flow_id"] = np.where(o["flow_id"] != R.FLOW_NONE,
                                    order[np.minimum(o["flow_id"], len(order) - 1)], R.FLOW_NONE)
            assert v[smp].tobytes() == o.tobytes(), b
    rebuilds = ctx.flows_rebuilds - rebuilds0
    ctx.close()
    host_us, dev_us = np.array(host_us), np.array(dev_us)
    print(f"churn at 1M tcbs, 1000 removed + 1000 added per burst: host median "
          f"{np.median(host_us):.0f} us (max {host_us.max():.0f}), commit on the GPU median "
          f"{np.median(dev_us):.0f} us (max {dev_us.max():.0f}); whole-table rebuilds {rebuilds}")
    assert rebuilds == 0  # steady churn never rebuilds
    assert np.median(host_us) + np.median(dev_us) < 1800, (np.median(host_us), np.median(dev_us))


def test_flows_sync_leaves_other_streams_running(torch_dev):
    """rxg_flows_sync waits for its own context's bursts only: queued work on
    another stream (not this context's) is still running when it returns"""
    torch, dev = torch_dev
    cfg = rxdist.gen_cfg("cfg2")
    udp, tcb = R.gen_flows(cfg)
    ctx = R.Context(0)
    ctx.flows_sync(udp, tcb)
    other = torch.cuda.Stream(dev)
    a = torch.empty(1 << 28, dtype=torch.uint8, device=dev)
    b = torch.empty_like(a)
    torch.cuda.synchronize(dev)
    with torch.cuda.stream(other):
        for _ in range(400):  # ~ tens of ms of copies
            b.copy_(a)
    t0 = time.perf_counter()
    ctx.flows_sync(udp, tcb)
    el = time.perf_counter() - t0
    busy = not other.query()
    torch.cuda.synchronize(dev)
    ctx.close()
    assert busy, f"flows_sync returned only after the other stream drained ({el * 1e3:.1f} ms)"


def test_api_restores_the_current_device(torch_dev):
    """every call leaves the calling thread on its own current device (with
    one GPU the context's device is the only one: the check still runs the
    save/restore path)"""
    torch, dev = torch_dev
    n = torch.cuda.device_count()
    other = 1 if n > 1 else 0
    torch.cuda.set_device(other)
    ctx = R.Context(0, max_pkts=1024, max_bytes=1 << 20)
    cfg = rxdist.gen_cfg("cfg2")
    udp, tcb = R.gen_flows(cfg)
    ctx.flows_sync(udp, tcb)
    assert torch.cuda.current_device() == other
    pk, off, ln = R.gen_host(cfg, 0, 100, 6)
    ctx.classify(pk, off, ln, 6)
    assert torch.cuda.current_device() == other
    ctx.flows_add(udp[:1], None)
    ctx.flow_counts()
    assert torch.cuda.current_device() == other
    ctx.close()
    assert torch.cuda.current_device() == other
    torch.cuda.set_device(0)


def test_count_stream_65536_flows_one_output_buffer(torch_dev):
    """exactly 65536 flows (2-B count indices, flow 65535's index
    is all ones), counts on a second stream, ONE verdict buffer reused by every
    burst, frames of flow 65535 in each: the counts are exact (the slab pass
    never reads verdicts a later burst may be rewriting)"""
    torch, dev = torch_dev
    nu = 65536
    udp = np.zeros(nu, R.UDP_SOCK_DTYPE)
    udp["localip"] = L
    udp["localport"] = (np.arange(nu) & 0xFFFF).astype(np.uint16)  # every raw port
    udp["protocol"] = 17
    ctx = R.Context(0)
    ctx.flows_sync(udp, None)
    n = 1 << 20
    rng = np.random.default_rng(7)
    ports = rng.integers(0, nu, n).astype(np.uint16)
    ports[::97] = 0xFFFF  # flow 65535: port raw 0xFFFF
    fr = np.zeros((n, 64), np.uint8)
    base = np.frombuffer(F.udp_frame("10.0.0.1", 5555, "192.168.100.77", 1, b"x" * 14), np.uint8)
    fr[:, :len(base)] = base
    fr[:, 36:38] = ports.view(np.uint8).reshape(n, 2)
    stream = torch.cuda.current_stream(dev)
    cs = torch.cuda.Stream(dev)
    d_pk = torch.from_numpy(np.concatenate([fr.reshape(-1), np.zeros(64, np.uint8)])).to(dev)
    d_off = torch.arange(n, dtype=torch.int32, device=dev)
    d_ln = torch.full((n,), len(base), dtype=torch.int16, device=dev)
    out = torch.empty(n * 16, dtype=torch.uint8, device=dev)
    cnt = torch.zeros(nu, dtype=torch.int64, device=dev)
    bursts = 12
    for _ in range(bursts):
        ctx.classify_dev(d_pk, d_off, d_ln, n, 6, 64, out, cnt, stream=stream.cuda_stream,
                         count_stream=cs.cuda_stream)
    stream.wait_stream(cs)
    torch.cuda.synchronize(dev)
    v = out.cpu().numpy().view(R.VERDICT_DTYPE)
    assert np.all(v["rc"] == 0) and np.array_equal(v["flow_id"], ports.astype(np.uint32))
    want = np.bincount(ports, minlength=nu).astype(np.uint64) * bursts
    assert np.array_equal(cnt.cpu().numpy().view(np.uint64), want)
    ctx.close()


def test_ctx_counts_allreduce_twice_keeps_totals(torch_dev):
    """the context's counts after repeated all-reduces are the
    running totals (a one-rank communicator here: the only group one GPU can
    form; the delta logic is the same at N ranks)"""
    torch, dev = torch_dev
    cfg = rxdist.gen_cfg("cfg2")
    udp, tcb = R.gen_flows(cfg)
    pk, off, ln = R.gen_host(cfg, 0, 5000, 6)
    ctx = R.Context(0, max_pkts=8192, max_bytes=1 << 22)
    ctx.flows_sync(udp, tcb)
    g = R.Group(0, 1, 0, R.group_id())
    want = O.Tables(udp, tcb).classify(pk, off, ln, 6, counts=True)[1]
    ctx.classify(pk, off, ln, 6)
    ctx.counts_allreduce(g)
    assert np.array_equal(ctx.flow_counts(), want)
    ctx.classify(pk, off, ln, 6)
    ctx.classify(pk, off, ln, 6)
    ctx.counts_allreduce(g)
    assert np.array_equal(ctx.flow_counts(), 3 * want)
    ctx.counts_reset()
    assert not ctx.flow_counts().any()
    g.close()
    ctx.close()


def test_udp_churn_small_socket_set(torch_dev):
    """<= 1024 sockets: the lane kernel's LDS copies (compact table, port
    window) follow every socket opened, rebound and closed; verdicts bit for
    bit against the oracle after each step"""
    torch, dev = torch_dev
    rng = np.random.default_rng(3)
    ctx = R.Context(0, max_pkts=4096, max_bytes=1 << 20)
    cfg = rxdist.gen_cfg("cfg2", n_udp=600)
    udp, _ = R.gen_flows(cfg)
    ctx.flows_sync(udp, None)
    live = {i: tuple(udp[i]) for i in range(len(udp))}
    seq = {i: i for i in live}
    nseq = len(udp)
    pk, off, ln = R.gen_host(cfg, 0, 3000, 6)
    for step in range(30):
        op = step % 3
        if op == 0:
            s = np.zeros(20, R.UDP_SOCK_DTYPE)
            s["localip"] = np.where(rng.random(20) < 0.8, L, R.ip_raw("10.1.1.1"))
            s["localport"] = np.array([R.port_raw(int(p)) for p in 20000 + rng.integers(0, 700, 20)],
                                      np.uint16)
            s["protocol"] = 17
            uid, _, _ = ctx.flows_add(s, None)
            for k, fid in enumerate(uid):
                live[int(fid)] = tuple(s[k])
                seq[int(fid)] = nseq
                nseq += 1
        elif op == 1:
            gone = rng.choice(list(live), 20, replace=False)
            ctx.flows_remove(gone, None)
            for fid in gone:
                del live[int(fid)], seq[int(fid)]
        else:
            fid = int(rng.choice(list(live)))
            s = np.zeros(1, R.UDP_SOCK_DTYPE)
            s[0] = (L, R.port_raw(int(20000 + rng.integers(0, 700))), 17, 0)
            ctx.flows_update_udp(fid, s[0])
            live[fid] = tuple(s[0])
        got = ctx.classify(pk, off, ln, 6)
        order = sorted(live, key=lambda i: seq[i])
        u = np.zeros(len(order), R.UDP_SOCK_DTYPE)
        for k, fid in enumerate(order):
            u[k] = live[fid]
        want = O.Tables(u, np.zeros(0, R.TCB_DTYPE)).classify(pk, off, ln, 6)
        m = want["flow_id"] != R.FLOW_NONE
        want["flow_id"][m] = np.array(order, np.uint32)[want["flow_id"][m]]
        assert got.tobytes() == want.tobytes(), step
    ctx.close()


def test_counts_move_with_the_id_space_tables_intact(torch_dev):
    """every rxg_flows_add grows the TCP id space, so the context's own count
    vector moves (counts_layout) in the commit of the next burst; that burst's
    kernel must count into the new vector.  Regression: the pointer was taken
    before the commit, so the kernel added into the freed vector, whose memory
    the same commit could hand to the grown TCP table (seen as +1 words in the
    device table and tcbs found as their listener).  After each burst: the
    device table equals the host image word for word, the verdicts equal the
    model's, and the counts equal the delivered frames per flow"""
    ctx = R.Context(0, max_pkts=4096, max_bytes=1 << 20)
    lis = np.zeros(1, R.TCB_DTYPE)
    lis[0] = (0, L, 0, P9999, R.TCP_STATUS_LISTEN)
    ctx.flows_sync(None, lis)
    want_counts = {0: 0}
    keys = []
    for k in range(40):
        t = np.zeros(1, R.TCB_DTYPE)
        cip = f"10.0.{k // 200}.{1 + k % 200}"
        t[0] = (R.ip_raw(cip), L, R.port_raw(40000 + k), P9999, 4)
        _, tid, _ = ctx.flows_add(None, t)
        keys.append((cip, 40000 + k, int(tid[0])))
        frames, ids = [], []
        for cip_, cport, fid in keys:
            frames.append(F.tcp_frame(cip_, cport, "192.168.100.77", 9999, b"x" * 10))
            ids.append(fid)
        frames.append(F.tcp_frame("10.9.9.9", 1234, "192.168.100.77", 9999, b"", flags=0x02))
        ids.append(0)  # no tcb: the listener
        buf, off, lens = F.pack_frames(frames, 6)
        got = ctx.classify(buf, off, lens, 6)
        assert list(got["flow_id"]) == ids and np.all(got["rc"] == 0), k
        for fid in ids:
            want_counts[fid] = want_counts.get(fid, 0) + 1
        hd, hi = R.ft_dump(ctx._h, 1, False)
        dd, di = R.ft_dump(ctx._h, 1, True)
        assert np.array_equal(hd, dd), (k, np.nonzero(hd != dd)[0][:8])
        c = ctx.flow_counts()
        nu = ctx.num_udp_ids
        assert all(int(c[nu + fid]) == n for fid, n in want_counts.items()), k
    ctx.close()


def test_reused_id_counts_only_its_own_frames(torch_dev):
    """a removed block's id is handed out again by the next add;
    the new block's context count must hold only its own frames, not the
    removed block's (the commit zeroes the counts of removed ids)"""
    ctx = R.Context(0, max_pkts=4096, max_bytes=1 << 20)
    lis = np.zeros(1, R.TCB_DTYPE)
    lis[0] = (0, L, 0, P9999, R.TCP_STATUS_LISTEN)
    t = np.zeros(2, R.TCB_DTYPE)
    t[0] = (R.ip_raw("10.0.0.1"), L, R.port_raw(40001), P9999, 4)
    t[1] = (R.ip_raw("10.0.0.2"), L, R.port_raw(40002), P9999, 4)
    ctx.flows_sync(None, np.concatenate([lis, t]))
    fr = [F.tcp_frame("10.0.0.1", 40001, "192.168.100.77", 9999, b"a" * 20)] * 7 + \
         [F.tcp_frame("10.0.0.2", 40002, "192.168.100.77", 9999, b"b" * 20)] * 3
    buf, off, lens = F.pack_frames(fr, 6)
    ctx.classify(buf, off, lens, 6)
    c = ctx.flow_counts()
    nu = ctx.num_udp_ids
    assert int(c[nu + 1]) == 7 and int(c[nu + 2]) == 3
    ctx.flows_remove(None, [1])
    nt = np.zeros(1, R.TCB_DTYPE)
    nt[0] = (R.ip_raw("10.0.0.9"), L, R.port_raw(40009), P9999, 4)
    _, tid, _ = ctx.flows_add(None, nt)
    assert int(tid[0]) == 1  # the freed id, reused
    fr2 = [F.tcp_frame("10.0.0.9", 40009, "192.168.100.77", 9999, b"c" * 20)] * 2
    buf, off, lens = F.pack_frames(fr2, 6)
    got = ctx.classify(buf, off, lens, 6)
    assert list(got["flow_id"]) == [1, 1]
    c = ctx.flow_counts()
    nu = ctx.num_udp_ids
    assert int(c[nu + 1]) == 2, c  # its own two frames only
    assert int(c[nu + 2]) == 3
    ctx.close()


def test_close_after_the_burst_stream_is_destroyed(torch_dev):
    """the usual teardown order — synchronise, destroy the stream
    the last burst ran on, then close the context — must not touch the
    destroyed stream (rxg_close records nothing on it)"""
    import ctypes as C
    torch, dev = torch_dev
    hip = C.CDLL("libamdhip64.so")
    st = C.c_void_p()
    assert hip.hipStreamCreate(C.byref(st)) == 0
    cfg = rxdist.gen_cfg("cfg2")
    udp, tcb = R.gen_flows(cfg)
    ctx = R.Context(0)
    ctx.flows_sync(udp, tcb)
    n = 4096
    pk = torch.empty(n * 64 + 64, dtype=torch.uint8, device=dev)
    off = torch.empty(n, dtype=torch.int32, device=dev)
    ln = torch.empty(n, dtype=torch.int16, device=dev)
    out = torch.empty(n * 16, dtype=torch.uint8, device=dev)
    R.gen_dev(cfg, 0, n, pk, off, ln, 6)
    torch.cuda.synchronize(dev)
    for _ in range(3):
        ctx.classify_dev(pk, off, ln, n, 6, 64, out, None, stream=st.value)
    assert hip.hipStreamSynchronize(st) == 0
    assert hip.hipStreamDestroy(st) == 0
    ctx.close()  # must neither crash nor fail
    v = out.cpu().numpy().view(R.VERDICT_DTYPE)
    assert np.all(v["rc"] <= 1)


def test_workspace_growth_leaves_other_streams_running(torch_dev):
    """a burst that grows the context's count workspace (slab path: > 8192
    flows, a larger burst than any before) frees and reallocates it in stream
    order: queued work on another stream is still running when the burst call
    returns, and the burst's counts are exact"""
    torch, dev = torch_dev
    cfg = rxdist.gen_cfg("cfg4")
    udp, tcb = R.gen_flows(cfg)
    ctx = R.Context(0)
    ctx.flows_sync(udp, tcb)
    n0, n1 = 1 << 12, 1 << 16
    pk = torch.empty(n1 * cfg.slot_bytes + 64, dtype=torch.uint8, device=dev)
    off = torch.empty(n1, dtype=torch.int32, device=dev)
    ln = torch.empty(n1, dtype=torch.int16, device=dev)
    out = torch.empty(n1 * 16, dtype=torch.uint8, device=dev)
    cnt = torch.zeros(ctx.num_flows, dtype=torch.int64, device=dev)
    R.gen_dev(cfg, 0, n1, pk, off, ln, 6)
    s = torch.cuda.current_stream(dev)
    ctx.classify_dev(pk, off, ln, n0, 6, 0, out, cnt, stream=s.cuda_stream)  # small workspace
    torch.cuda.synchronize(dev)
    other = torch.cuda.Stream(dev)
    a = torch.empty(1 << 28, dtype=torch.uint8, device=dev)
    b = torch.empty_like(a)
    torch.cuda.synchronize(dev)
    with torch.cuda.stream(other):
        for _ in range(400):
            b.copy_(a)
    cnt.zero_()
    ctx.classify_dev(pk, off, ln, n1, 6, 0, out, cnt, stream=s.cuda_stream)  # grows it
    busy = not other.query()
    torch.cuda.synchronize(dev)
    assert busy, "the growing burst waited for another stream's work"
    v = out[:n1 * 16].cpu().numpy().view(R.VERDICT_DTYPE)
    ok = v["rc"] == 0
    nu = len(udp)
    idx = np.where(v["cls"][ok] == R.CLS_UDP, v["flow_id"][ok], nu + v["flow_id"][ok].astype(np.int64))
    want = np.bincount(idx, minlength=ctx.num_flows).astype(np.uint64)
    assert np.array_equal(cnt.cpu().numpy().view(np.uint64), want)
    ctx.close()
