"""Incremental flow-table changes (rxg_flows_add / remove / update), host side.

The reference creates a tcb on every SYN (tcp_stream_create + LL_ADD,
tcp.c:3-52), binds and listens sockets in place (common.c:342-386) and frees
blocks on the last ACK and on close (tcp.c:321, common.c:620,660); lookups are
first-match walks of the head-inserted lists (common.c:31-55, 97-108), i.e.
the newest block with the key wins, and the listener pass takes the newest
LISTEN block on the port.  These tests churn a control-plane-only context
(RXG_HOST_ONLY: the same host tables the device copies) and check every
lookup against two references: a plain model of the lists, and the oracle's
list scans over the live blocks in creation order (its index mapped to the
block's stable id).  The device side is tests/test_gpu_churn.py."""
import numpy as np
import pytest

import oracle_bind as O
import rxgpu as R

LISTEN, EST = R.TCP_STATUS_LISTEN, R.TCP_STATUS_ESTABLISHED


class Model:
    """the reference's lists: blocks in creation order, lookups newest-first"""

    def __init__(self):
        self.udp = {}  # stable id -> [seq, (ip, port, proto)]
        self.tcp = {}  # stable id -> [seq, (sip, dip, sport, dport, status)]
        self.seq = 0

    def add_udp(self, fid, sock):
        self.seq += 1
        self.udp[fid] = [self.seq, tuple(int(x) for x in sock)[:3]]

    def add_tcp(self, fid, t):
        self.seq += 1
        self.tcp[fid] = [self.seq, tuple(int(x) for x in t)]

    def lookup_udp(self, dip, dport):
        best = None
        for fid, (sq, (ip, port, proto)) in self.udp.items():
            if ip == dip and port == dport and proto == 17 and (best is None or sq > best[0]):
                best = (sq, fid)
        return R.FLOW_NONE if best is None else best[1]

    def lookup_tcp(self, sip, dip, sport, dport):
        best = None
        for fid, (sq, (a, b, c, d, st)) in self.tcp.items():
            if (a, b, c, d) == (sip, dip, sport, dport) and (best is None or sq > best[0]):
                best = (sq, fid)
        if best is None:
            for fid, (sq, (a, b, c, d, st)) in self.tcp.items():
                if d == dport and st == LISTEN and (best is None or sq > best[0]):
                    best = (sq, fid)
        return R.FLOW_NONE if best is None else best[1]

    def oracle(self):
        """the oracle's tables over the live blocks in creation order, and the
        stable id of each of its indices"""
        uo = sorted(self.udp.items(), key=lambda kv: kv[1][0])
        to = sorted(self.tcp.items(), key=lambda kv: kv[1][0])
        u = np.zeros(len(uo), R.UDP_SOCK_DTYPE)
        for k, (fid, (_, key)) in enumerate(uo):
            u[k] = key + (0,)
        t = np.zeros(len(to), R.TCB_DTYPE)
        for k, (fid, (_, key)) in enumerate(to):
            t[k] = key
        return O.Tables(u, t), [fid for fid, _ in uo], [fid for fid, _ in to]


def _sock(ip, port, proto=17):
    a = np.zeros(1, R.UDP_SOCK_DTYPE)
    a[0] = (ip, port, proto, 0)
    return a


def _tcb(sip, dip, sport, dport, st):
    a = np.zeros(1, R.TCB_DTYPE)
    a[0] = (sip, dip, sport, dport, st)
    return a


def _check_all(ctx, m, probes_u, probes_t):
    tb, umap, tmap = m.oracle()
    for dip, dport in probes_u:
        want = m.lookup_udp(dip, dport)
        got = ctx.lookup_udp(dip, dport)
        assert got == want, ("udp", dip, dport, got, want)
        o = tb.lookup_udp(dip, dport)
        assert (R.FLOW_NONE if o == R.FLOW_NONE else umap[o]) == want
    for key in probes_t:
        want = m.lookup_tcp(*key)
        got = ctx.lookup_tcp(*key)
        assert got == want, ("tcp", key, got, want)
        o = tb.lookup_tcp(*key)
        assert (R.FLOW_NONE if o == R.FLOW_NONE else tmap[o]) == want


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_churn_matches_list_walks(seed):
    """random add / remove / rebind / listen over a small key space, so
    duplicate keys (newest wins, the next older one after a remove), several
    listeners per port, id reuse and socket addresses off the port table's
    address all occur; every lookup checked after every step"""
    rng = np.random.default_rng(seed)
    ctx = R.Context(R.HOST_ONLY)
    m = Model()
    ips = [R.ip_raw(x) for x in ("192.168.100.77", "192.168.100.77", "10.9.9.9", "0.0.0.0")]
    ports = [R.port_raw(p) for p in (7, 8, 9, 20000, 9999)]
    srcs = [R.ip_raw(x) for x in ("10.0.0.1", "10.0.0.2")]
    probes_u = [(ip, p) for ip in set(ips) for p in ports]
    probes_t = [(s, d, sp, dp) for s in srcs + [0] for d in set(ips)
                for sp in ports[:2] + [0] for dp in ports[3:]]
    for step in range(300):
        op = rng.integers(0, 6)
        if op == 0 or not m.udp:
            s = _sock(ips[rng.integers(len(ips))], ports[rng.integers(len(ports))],
                      17 if rng.random() < 0.95 else 6)
            uid, _, _ = ctx.flows_add(s, None)
            m.add_udp(int(uid[0]), s[0])
        elif op == 1 or not m.tcp:
            st = LISTEN if rng.random() < 0.3 else EST
            t = _tcb(srcs[rng.integers(2)] if st == EST else 0, ips[rng.integers(len(ips))],
                     ports[rng.integers(2)] if st == EST else 0, ports[3 + rng.integers(2)], st)
            _, tid, _ = ctx.flows_add(None, t)
            m.add_tcp(int(tid[0]), t[0])
        elif op == 2:
            fid = int(rng.choice(list(m.udp)))
            ctx.flows_remove([fid], None)
            del m.udp[fid]
        elif op == 3:
            fid = int(rng.choice(list(m.tcp)))
            ctx.flows_remove(None, [fid])
            del m.tcp[fid]
        elif op == 4:  # nbind: same list position, new key
            fid = int(rng.choice(list(m.udp)))
            s = _sock(ips[rng.integers(len(ips))], ports[rng.integers(len(ports))])
            ctx.flows_update_udp(fid, s[0])
            m.udp[fid][1] = tuple(int(x) for x in s[0])[:3]
        else:  # nlisten / a state change: same position, status (and maybe key)
            fid = int(rng.choice(list(m.tcp)))
            sq, (a, b, c, d, st) = m.tcp[fid]
            st2 = LISTEN if st != LISTEN else EST
            if rng.random() < 0.3:
                d = ports[3 + rng.integers(2)]
            t = _tcb(a, b, c, d, st2)
            ctx.flows_update_tcb(fid, t[0])
            m.tcp[fid][1] = (a, b, c, d, st2)
        _check_all(ctx, m, probes_u, probes_t)
    ctx.close()


def test_ids_are_stable_and_reused():
    ctx = R.Context(R.HOST_ONLY)
    udp = np.zeros(3, R.UDP_SOCK_DTYPE)
    for k in range(3):
        udp[k] = (R.ip_raw("1.2.3.4"), R.port_raw(100 + k), 17, 0)
    ctx.flows_sync(udp, None)
    assert [ctx.lookup_udp(R.ip_raw("1.2.3.4"), R.port_raw(100 + k)) for k in range(3)] == [0, 1, 2]
    ctx.flows_remove([1], None)
    assert ctx.lookup_udp(R.ip_raw("1.2.3.4"), R.port_raw(101)) == R.FLOW_NONE
    assert ctx.lookup_udp(R.ip_raw("1.2.3.4"), R.port_raw(102)) == 2  # not renumbered
    uid, _, moved = ctx.flows_add(_sock(R.ip_raw("1.2.3.4"), R.port_raw(555)), None)
    assert uid[0] == 1 and not moved  # the freed id, the layout unchanged
    uid, _, _ = ctx.flows_add(_sock(R.ip_raw("1.2.3.4"), R.port_raw(556)), None)
    assert uid[0] == 3 and ctx.num_udp_ids == 4
    with pytest.raises(R.RxgError):
        ctx.flows_remove([7], None)  # no such id
    ctx.close()


def test_count_layout_moves_when_the_udp_ids_grow():
    ctx = R.Context(R.HOST_ONLY)
    ctx.flows_sync(_sock(1, 2), _tcb(3, 4, 5, 6, EST))
    assert (ctx.num_udp_ids, ctx.num_flows) == (1, 2)
    _, _, moved = ctx.flows_add(_sock(1, 3), None)
    assert moved and (ctx.num_udp_ids, ctx.num_flows) == (2, 3)
    _, _, moved = ctx.flows_add(None, _tcb(3, 4, 5, 7, EST))
    assert not moved and ctx.num_flows == 4
    ctx.close()


def test_growth_and_bulk_churn_at_scale():
    """100K tcbs added one batch at a time from an empty table (rebuilt as it
    passes load 1/2), then 40% removed: lookups stay exact and the rebuilds
    stay logarithmic in the size"""
    ctx = R.Context(R.HOST_ONLY)
    rng = np.random.default_rng(5)
    n = 100000
    t = np.zeros(n, R.TCB_DTYPE)
    t["sip"] = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    t["dip"] = R.ip_raw("192.168.100.77")
    t["sport"] = rng.integers(0, 2**16, n).astype(np.uint16)
    t["dport"] = R.port_raw(9999)
    t["status"] = EST
    ids = []
    for k in range(0, n, 10000):
        ids.append(ctx.flows_add(None, t[k:k + 10000])[1])
    ids = np.concatenate(ids)
    assert np.array_equal(ids, np.arange(n))
    assert ctx.flows_rebuilds <= 20
    gone = rng.choice(n, 40000, replace=False)
    ctx.flows_remove(None, gone)
    alive = np.ones(n, bool)
    alive[gone] = False
    for k in rng.choice(n, 3000, replace=False):
        got = ctx.lookup_tcp(int(t["sip"][k]), int(t["dip"][k]), int(t["sport"][k]),
                             int(t["dport"][k]))
        # (random 4-tuples: a duplicate key resolves to its newest live block)
        same = np.nonzero((t["sip"] == t["sip"][k]) & (t["sport"] == t["sport"][k]) & alive)[0]
        assert got == (same.max() if len(same) else R.FLOW_NONE), k
    ctx.close()
