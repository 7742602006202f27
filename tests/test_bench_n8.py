"""The N = 8 bench line, built on CPU by 8 gloo ranks.

The driver's 8-GPU run (`bench.py --gpus 8`, one rank per GPU over RCCL) has
never been run by this repository: no 8-GPU box is ours to launch.  What can
be rehearsed here is every step of it that does not touch a GPU, with the
same code bench.py runs:

  - the launcher starts 8 rank processes and their gloo rendezvous sees 8
    (bench.py --gpus 8 on this GPU-less box: every rank then exits 4);
  - bench.gather_rank_stats: the per-rank wall / kernel-stream / all-reduce
    times and frames, and the max over ranks that `value` divides by, over 8
    gloo ranks;
  - bench.burst_digest in split mode: each rank holds a shard of one burst
    (here BASELINE configs[0], cfg1's 100,000 frames, partitioned by frame
    index; its verdicts from the oracle, the checker, standing in for each
    rank's GPU) and the ranks' partial frame digests are summed over gloo and
    compared with the golden digest of the whole burst (digest_ok);
  - bench.build_line + compact_line on rank 0: the line with an 8-entry
    per_rank for each of the four workloads stays under LINE_MAX, parses, and
    carries ranks.n = 8 and ranks.rccl_nranks (the count the RCCL
    communicator reports on the real run; None here, where gloo stands in).
"""
import importlib.util
import json
import os
import socket
import subprocess
import sys

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle_bind as O
import rxdist
import rxgpu as R

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")
WORLD = 8


def _bench():
    spec = importlib.util.spec_from_file_location("bench_n8", BENCH)
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _head(name, w, n_all, per_rank, el, dg, steps):
    """a workload's result as run_workload returns it, with this rank set's
    gathered per_rank and time (the GPU-measured fields are stand-ins)"""
    return dict(workload=name, desc=w["desc"], frames_per_step=n_all, nflows=1024,
                mpps=n_all * steps / el / 1e6, gbps=86 * n_all * steps / el / 1e9,
                ms_per_step=el / steps * 1e3, kernel_ms_avg=0.2301, counts_ok=True,
                counts_match=True, allreduce_ms=0.0123, allreduce_bytes=8 * 1024,
                per_rank=per_rank, parity=dict(checked=4096 * WORLD, mismatches=0),
                digest=dg,
                roofline=dict(bound="hbm", achieved=6200.0, peak=8000.0, unit="GB/s", frac=0.775,
                              traffic=None, kernel=dict(name="rx_classify_lane_kernel",
                                                        median_ms=0.2301, frac=0.775)))


def _rank(rank, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        B = _bench()
        w = rxdist.WORKLOADS["cfg1"]
        cfg = rxdist.gen_cfg("cfg1")
        pk, off, ln = R.gen_host(cfg, 0, w["n"], w["unit_log2"])
        udp, tcb = R.gen_flows(cfg)
        mine = np.arange(rank, w["n"], WORLD, dtype=np.int64)  # this rank's shard
        v = O.Tables(udp, tcb).classify(pk, off[mine], ln[mine], w["unit_log2"])
        out = torch.from_numpy(np.frombuffer(v.tobytes(), np.uint8).copy())
        n = len(mine)
        dg = B.burst_digest("cfg1", out, n, mine, None, 1, rank, WORLD, "split")
        steps = 50
        el = (0.2300 + 0.0002 * rank) * 1e-3 * steps  # stand-in timed region, seconds
        per_rank, el_max = B.gather_rank_stats(WORLD, el, steps, 0.229 + 0.0001 * rank,
                                               0.0123, n)
        if rank == 0:
            names = ["cfg2", "cfg3", "cfg4", "cfg5"]
            res = {nm: _head(nm, rxdist.WORKLOADS[nm], n * WORLD, per_rank, el_max, dg, steps)
                   for nm in names}
            line = B.build_line(names, res, steps, 5, 200.0, WORLD, 0,
                                "gloo (stand-in for rccl)", None)
            short = B.compact_line(line)
            q.put((rank, dict(line=line, short=json.dumps(short, separators=(",", ":")),
                              el_max=el_max, limit=B.LINE_MAX)))
        else:
            q.put((rank, dict(digest=dg)))
    finally:
        dist.destroy_process_group()


def test_eight_rank_line_on_cpu():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_rank, args=(r, port, q)) for r in range(WORLD)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=300) for _ in range(WORLD))
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    r0 = got[0]
    line, short = r0["line"], json.loads(r0["short"])
    assert len(r0["short"]) < r0["limit"], len(r0["short"])
    print("N = 8 compact line:", len(r0["short"]), "bytes")
    assert "dropped" not in short, short.get("dropped")
    assert line["n_gpus"] == WORLD and len(line["per_rank"]) == WORLD
    assert [p["rank"] for p in line["per_rank"]] == list(range(WORLD))
    assert sum(p["frames"] for p in line["per_rank"]) == 100000
    # value divides by the slowest rank's time
    assert abs(r0["el_max"] - (0.2300 + 0.0002 * (WORLD - 1)) * 1e-3 * 50) < 1e-12
    assert short["ranks"]["n"] == WORLD and "rccl_nranks" in short["ranks"]
    assert abs(short["ranks"]["ms_per_step_max"] - 0.2314) < 1e-4
    # the split digest: 8 partial sums of one golden burst
    assert short["digest_ok"] is True, line["digest"]
    assert line["digest"]["frames"] == 100000
    for r in range(1, WORLD):
        assert got[r]["digest"]["frame_digest"] == line["digest"]["frame_digest"]
    for nm in ("cfg3", "cfg4", "cfg5"):
        assert nm in short


def test_launcher_starts_eight_ranks():
    """bench.py --gpus 8 with no launcher: 8 processes, a gloo rendezvous of
    8, then each rank fails loudly (no GPU here; no CPU path to measure)"""
    if torch.cuda.device_count():
        import pytest
        pytest.skip("GPU present: the spawn is exercised by the real bench")
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, BENCH, "--gpus", "8", "--backend", "gloo", "--steps", "1"],
                       env=env, capture_output=True, text=True, timeout=400)
    err = r.stderr
    assert "bench: launched 8 ranks" in err, err
    for k in range(WORLD):
        assert f"bench: rank {k}: rendezvous ok, all_reduce saw 8 ranks" in err, err
    assert "bench: rank exit codes [4, 4, 4, 4, 4, 4, 4, 4]" in err, err
    assert r.returncode == 4 and r.stdout.strip() == ""
