"""Whole-burst verdict digests (tests/golden/digests.json, made by
tests/golden/make_digests.py from the oracle over every frame of each BASELINE
config's burst).  SURVEY §4 item 4 / §8(c): bit-exact verdict arrays plus
SHA-256 — every verdict of every full-size burst, not a sample; the
per-frame producers are udp.c:14-19 and tcp.c:349-371.

CPU: the numpy and torch forms of the order-free frame digest agree; the
oracle reproduces the committed digests of the configs it can rerun in
seconds (cfg1, cfg2 sample-free at 100K/16M frames would take ~20 s: cfg1 and
cfg3 are rerun).  GPU: each config's whole burst classified on the device
hashes to the committed digests (verdicts and per-flow counts)."""
import numpy as np
import pytest

import digest as D
import rxdist
import rxgpu as R

GOLD = D.load_golden()


def test_frame_digest_numpy_equals_torch():
    import torch
    rng = np.random.default_rng(0)
    v = rng.integers(0, 256, (5000, 16), dtype=np.uint8)
    idx = rng.integers(0, 1 << 40, 5000).astype(np.uint64)
    a = D.frame_digest_np(idx, v)
    b = D.frame_digest_torch(torch.from_numpy(idx.astype(np.int64)), torch.from_numpy(v.reshape(-1)))
    assert a == b
    # order-free: any partition into shards adds up to the whole
    parts = np.array_split(rng.permutation(5000), 3)
    tot = sum(D.frame_digest_np(idx[p], v[p]) for p in parts) & D._M64
    assert tot == a


@pytest.mark.parametrize("name", ["cfg1", "cfg3"])
def test_oracle_reproduces_committed_digest(name):
    import make_digests_path  # noqa: F401  (puts tests/golden on sys.path)
    import make_digests as M
    r = M.digest_config(name, threads=8)
    g = GOLD[name]
    for k in ("frames", "verdict_sha256", "frame_digest", "counts_sha256", "counted"):
        assert r[k] == g[k], (name, k, r[k], g[k])


def test_golden_covers_every_config():
    assert set(GOLD) == {"cfg1", "cfg2", "cfg3", "cfg4", "cfg5"}
    for name, g in GOLD.items():
        assert g["frames"] == rxdist.WORKLOADS[name]["n"], name
        assert g["counted"] == g["rc"].get("0", 0), name  # every rc-0 frame counted once


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["cfg1", "cfg2", "cfg3", "cfg4", "cfg5"])
def test_gpu_whole_burst_matches_golden_digest(name):
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a GPU (no fallback path exists)")
    dev = torch.device("cuda", 0)
    w = rxdist.WORKLOADS[name]
    cfg = rxdist.gen_cfg(name)
    n, ul = w["n"], w["unit_log2"]
    udp, tcb = R.gen_flows(cfg)
    g = GOLD[name]
    with R.Context(0) as ctx:
        ctx.flows_sync(udp, tcb)
        d_pk = torch.empty(n * cfg.slot_bytes + 64, dtype=torch.uint8, device=dev)
        d_off = torch.empty(n, dtype=torch.int32, device=dev)
        d_ln = torch.empty(n, dtype=torch.int16, device=dev)
        sh = torch.cuda.current_stream(dev).cuda_stream
        R.gen_dev(cfg, 0, n, d_pk, d_off, d_ln, ul, stream=sh)
        out = torch.empty(n * 16, dtype=torch.uint8, device=dev)
        cnt = torch.zeros(max(ctx.num_flows, 1), dtype=torch.int64, device=dev)
        ctx.classify_dev(d_pk, d_off, d_ln, n, ul, w["len_hint"], out, cnt, stream=sh)
        torch.cuda.synchronize(dev)
        fd = D.frame_digest_torch(torch.arange(n, dtype=torch.int64, device=dev), out)
        assert f"{fd:016x}" == g["frame_digest"], name
        assert D.sha256_bytes(out.cpu().numpy()) == g["verdict_sha256"], name
        c = cnt.cpu().numpy().view(np.uint64)[:ctx.num_flows]
        assert D.counts_sha256(c) == g["counts_sha256"], name
        del d_pk, out
        torch.cuda.empty_cache()


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["cfg1", "cfg2", "cfg3", "cfg4", "cfg5"])
def test_gpu_whole_burst_v8_matches_golden_digest(name):
    """rxg_classify_dev8 (8-B verdicts, counts on a second stream above 8192
    flows): every verdict of the full burst hashes to the oracle's projected
    digest, and the per-flow counts to the oracle's histogram"""
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a GPU (no fallback path exists)")
    dev = torch.device("cuda", 0)
    w = rxdist.WORKLOADS[name]
    cfg = rxdist.gen_cfg(name)
    n, ul = w["n"], w["unit_log2"]
    udp, tcb = R.gen_flows(cfg)
    g = GOLD[name]
    with R.Context(0) as ctx:
        ctx.flows_sync(udp, tcb)
        d_pk = torch.empty(n * cfg.slot_bytes + 64, dtype=torch.uint8, device=dev)
        d_off = torch.empty(n, dtype=torch.int32, device=dev)
        d_ln = torch.empty(n, dtype=torch.int16, device=dev)
        st = torch.cuda.current_stream(dev)
        cs = torch.cuda.Stream(dev)
        R.gen_dev(cfg, 0, n, d_pk, d_off, d_ln, ul, stream=st.cuda_stream)
        out = torch.empty(n * 8, dtype=torch.uint8, device=dev)
        cnt = torch.zeros(max(ctx.num_flows, 1), dtype=torch.int64, device=dev)
        ctx.classify_dev8(d_pk, d_off, d_ln, n, ul, w["len_hint"], out, cnt, stream=st.cuda_stream,
                          count_stream=cs.cuda_stream)
        torch.cuda.synchronize(dev)
        assert D.sha256_bytes(out.cpu().numpy()) == g["verdict8_sha256"], name
        c = cnt.cpu().numpy().view(np.uint64)[:ctx.num_flows]
        assert D.counts_sha256(c) == g["counts_sha256"], name
        del d_pk, out
        torch.cuda.empty_cache()
