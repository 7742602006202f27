#!/usr/bin/env python3
"""bench.py — device-resident rx parse + checksum + flow-classify throughput.

Metric (BASELINE.json): Mpps + GB/s, device-resident, 64 B & 1500 B frames.
A "step" = one pass of the hot path (rxg_classify_dev: the fused gfx950
kernel) over one burst of synthetic frames already resident in HBM, plus at
N > 1 the per-flow count all-reduce (the path's only exchange).
Default workload = BASELINE configs[1] (64 B UDP, 1024 flows, 16M frames per
GPU); configs[2..4] are measured in the same run and reported under
"cfg3".."cfg5", BASELINE configs[0] (100K x 64 B UDP from a pcap, 1 flow)
under "cfg1".

N > 1 (one rank per GPU, weak scaling): every rank generates the GLOBAL burst
of N x n frames, RSS-splits it on its GPU (rxg_rss_split_dev) and gathers its
own shard (rxg_gather_dev) before the timed steps; a step classifies the shard
and all-reduces the per-flow counts over RCCL (rxg_counts_allreduce); value =
N x n frames / the max-over-ranks step time.  Every workload line carries a
"parity" field: a seeded sample of the run's verdicts checked bit for bit
against the oracle (the exit code is 3 if any differs).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload cfg2,cfg3]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
"""
from __future__ import annotations

import argparse
import ctypes as C
import glob
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "dpdk-tcp-udp_protocol_stack_amd")
sys.path.insert(0, PKG)


def _gpus_arg(argv):
    """--gpus N from the command line, read before anything touches the GPU"""
    for k, a in enumerate(argv):
        if a == "--gpus" and k + 1 < len(argv):
            return int(argv[k + 1])
        if a.startswith("--gpus="):
            return int(a.split("=", 1)[1])
    return 1


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _deadline_arg(argv):
    """--deadline S (seconds) from the command line; default from the
    workload list: 120 s + 120 s per workload (a healthy N-rank run of the
    default four workloads takes a few minutes at most)"""
    wl = "cfg2,cfg3,cfg4,cfg5"
    for k, a in enumerate(argv):
        if a == "--deadline" and k + 1 < len(argv):
            return float(argv[k + 1])
        if a.startswith("--deadline="):
            return float(a.split("=", 1)[1])
        if a == "--workload" and k + 1 < len(argv):
            wl = argv[k + 1]
        elif a.startswith("--workload="):
            wl = a.split("=", 1)[1]
    return 120.0 + 120.0 * len([w for w in wl.split(",") if w.strip()])


def stage(rank, what):
    """this rank's progress: a line on stderr, and (under launch_ranks) the
    rank's stage file, which the launcher prints if the run outlives its
    deadline, so a hang names the stage it stopped in"""
    print(f"bench: rank {rank}: stage {what}", file=sys.stderr, flush=True)
    d = os.environ.get("BENCH_STAGE_DIR")
    if d:
        try:
            with open(os.path.join(d, f"rank{rank}"), "w") as f:
                f.write(what)
        except OSError:
            pass


def launch_ranks(n: int, argv) -> int:
    """`bench.py --gpus N` with no launcher: start N rank processes of this
    script (one per GPU, RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set), as
    torch.distributed.run would, and exit with the worst child status.  Runs
    before torch or librxgpu is imported, so this process never touches the
    GPU (children are started, never exec'd).  Rank 0 prints the JSON line on
    the inherited stdout.  When a rank fails, the others get 60 s to finish
    and are then terminated (a peer stuck in a barrier would wait forever).
    The whole run has a wall-clock deadline (--deadline, default from the
    workload list): past it every rank still running is terminated (killed
    10 s later), each rank's last stage is printed, and the exit code is 124."""
    import shutil
    import subprocess
    import tempfile
    import time as _t
    deadline_s = _deadline_arg(argv)
    stage_dir = tempfile.mkdtemp(prefix="bench_stage_")
    env0 = dict(os.environ)
    env0.setdefault("MASTER_ADDR", "127.0.0.1")
    env0.setdefault("MASTER_PORT", str(_free_port()))
    env0["WORLD_SIZE"] = str(n)
    env0["LOCAL_WORLD_SIZE"] = str(n)
    env0["BENCH_STAGE_DIR"] = stage_dir
    env0.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    procs = []
    for r in range(n):
        env = dict(env0, RANK=str(r), LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv),
                                      env=env))
    print(f"bench: launched {n} ranks (pids {[p.pid for p in procs]}, "
          f"MASTER {env0['MASTER_ADDR']}:{env0['MASTER_PORT']}, deadline {deadline_s:.0f} s)",
          file=sys.stderr, flush=True)
    t_end = _t.monotonic() + deadline_s
    grace = None    # a rank failed: the others' time to finish
    kill_at = None  # terminated: SIGKILL for whoever is left at this time
    timed_out = False
    while True:
        rcs = [p.poll() for p in procs]
        if all(rc is not None for rc in rcs):
            break
        now = _t.monotonic()
        if not timed_out and now > t_end:
            timed_out = True
            for r, p in enumerate(procs):
                if p.poll() is None:
                    try:
                        with open(os.path.join(stage_dir, f"rank{r}")) as f:
                            st = f.read()
                    except OSError:
                        st = "(none reported: before the rendezvous)"
                    print(f"bench: deadline {deadline_s:.0f} s passed; rank {r} (pid {p.pid}) "
                          f"still running, last stage: {st}", file=sys.stderr, flush=True)
            grace = now  # terminate at once
        if grace is None and any(rc not in (None, 0) for rc in rcs):
            grace = now + 60.0
        if grace is not None and kill_at is None and now >= grace:
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            kill_at = now + 10.0
        if kill_at is not None and now > kill_at:
            for p in procs:
                if p.poll() is None:
                    p.kill()
            kill_at = float("inf")
        _t.sleep(0.2)
    shutil.rmtree(stage_dir, ignore_errors=True)
    rcs = [p.returncode for p in procs]
    print(f"bench: rank exit codes {rcs}", file=sys.stderr, flush=True)
    if timed_out:
        return 124
    bad = [rc for rc in rcs if rc != 0]
    return 0 if not bad else (bad[0] if bad[0] > 0 else 128 - bad[0])


if __name__ == "__main__":
    _n = _gpus_arg(sys.argv[1:])
    _ws = os.environ.get("WORLD_SIZE")
    if _n > 1 and _ws is None:
        sys.exit(launch_ranks(_n, sys.argv[1:]))
    if _ws is not None and int(_ws) != _n:
        print(f"bench: --gpus {_n} but the launcher started WORLD_SIZE={_ws} ranks; "
              "they must agree", file=sys.stderr, flush=True)
        sys.exit(2)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import rxdist  # noqa: E402
import rxgpu as R  # noqa: E402

COUNTS = True
CS_PRIORITY = 0  # torch stream priority of the count stream (--count-stream-priority)
CU_SPLIT = 0  # CUs reserved for the count stream (--cu-split; 0 = shared)
# above 8192 flows the per-flow counts are two passes after the classify kernel;
# on a second stream (rxg_classify_dev_cs) they overlap the next step's classify
COUNT_STREAM = True
TX = True
V8 = True  # also time the steps with 8-B verdicts (rxg_classify_dev8)
RAMP_MS = 200.0
RAMP_MAX_S = 15.0  # the adaptive part of the ramp stops here
JSON_OUT = sys.stdout
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level table)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


# ---------------------------------------------------------------------------
def collective_fn(group, nccl_group, nflows):
    """the path's one exchange, on stream `cs`: rxgpu.Group (RCCL through the
    C ABI) or, if that could not be opened, torch.distributed's RCCL"""
    def run(t, cs):
        if group is not None:
            group.allreduce(t, nflows, stream=cs.cuda_stream)
        else:
            with torch.cuda.stream(cs):
                torch.distributed.all_reduce(t, group=nccl_group)
    return run


def cu_split_streams(dev, n_count):
    """two streams on disjoint CUs (hipExtStreamCreateWithCUMask): the
    classify stream on all but n_count CUs, the count stream on those n_count.
    The slab pass's 1024-thread, 128-KiB-LDS blocks need a CU with nothing
    else on it, which the next burst's classify never leaves free (DESIGN §6,
    round 6); CUs of their own let the count of burst k run beside the
    classify of burst k+1.  Returns (classify stream, count stream) as torch
    ExternalStreams.  The streams live for the rest of the process (torch's
    allocator keeps them in its records of the tensors they used).
    n_count > 0: the count CUs spread one per 32-CU group (an XCD of MI355X,
    as HIP numbers CUs); n_count < 0: the last |n_count| CUs."""
    import ctypes as C
    path = [ln.split()[-1] for ln in open("/proc/self/maps") if "libamdhip64" in ln][0]
    hip = C.CDLL(path)  # the HIP runtime this process already uses (torch's, librxgpu's)
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    words = (ncu + 31) // 32
    made = []

    if n_count > 0:  # spread: CU 32g + 31 - j of group g, round robin
        groups = max(1, ncu // 32)
        count_cus = {32 * (j % groups) + 31 - j // groups for j in range(n_count)}
    else:
        count_cus = set(range(ncu + n_count, ncu))

    def make(cus):
        m = (C.c_uint32 * words)()
        for i in cus:
            m[i // 32] |= 1 << (i % 32)
        h = C.c_void_p()
        rc = hip.hipExtStreamCreateWithCUMask(C.byref(h), C.c_uint32(words), m)
        if rc != 0:
            raise RuntimeError(f"hipExtStreamCreateWithCUMask: {rc}")
        made.append(h)
        return torch.cuda.ExternalStream(h.value, device=dev)

    cls = make(sorted(set(range(ncu)) - count_cus))
    cnt = make(sorted(count_cus))
    return cls, cnt, lambda: torch.cuda.synchronize(dev)


def gather_rank_stats(world, el, steps, stream_ms, ar_ms, n):
    """N > 1, every rank: each rank's wall step, kernel-stream step,
    all-reduce time and frames (all_gather over the control plane, gloo), and
    the max over ranks of the timed region's wall time, which `value` divides
    by.  Returns (per_rank list, max wall seconds)."""
    mine = torch.tensor([el / max(steps, 1) * 1e3, stream_ms, ar_ms, float(n)], dtype=torch.float64)
    allr = [torch.zeros_like(mine) for _ in range(world)]
    torch.distributed.all_gather(allr, mine)
    per_rank = [dict(rank=r, ms_per_step=round(float(x[0]), 4),
                     stream_ms_per_step=round(float(x[1]), 4),
                     allreduce_ms=round(float(x[2]), 4), frames=int(x[3]))
                for r, x in enumerate(allr)]
    t = torch.tensor([el], dtype=torch.float64)
    torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    return per_rank, float(t.item())


def run_workload(name, ctx, rank, world, steps, warmup, dev, coll=None, parity_sample=4096,
                 oracle_threads=1, shard_mode="direct"):
    w = rxdist.WORKLOADS[name]
    cfg = rxdist.gen_cfg(name)
    ul = w["unit_log2"]
    udp, tcb = R.gen_flows(cfg)
    ctx.flows_sync(udp, tcb)
    nflows = len(udp) + len(tcb)
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream
    t_setup = time.perf_counter()
    pk, off, ln, n, gidx, gcfg = rxdist.build_shard(ctx, name, rank, world, dev, stream,
                                                    shard_mode)
    t_setup = time.perf_counter() - t_setup
    out = torch.empty(max(n, 1) * 16, dtype=torch.uint8, device=dev)
    counts = torch.zeros(max(nflows, 1), dtype=torch.int64, device=dev)
    frame_bytes = int(ln[:n].to(torch.int64).bitwise_and(0xFFFF).sum().item())
    alg_bytes = frame_bytes + 22 * n  # frame + off(4) + len(2) read + verdict(16) written
    # N > 1: step k's counts go to step_counts[k & 1]; the all-reduce runs on
    # the collective stream cs while step k+1's kernel runs, then adds into counts
    # the count stream only where the counts are separate passes (slab path,
    # R.SLAB_MIN_FLOWS flows and up); below that the classify kernel counts
    # itself and the stream would only add an event per step (~3 us of GPU
    # idle between bursts, r02j)
    use_cs = COUNT_STREAM and COUNTS and nflows >= R.SLAB_MIN_FLOWS
    # (CS_PRIORITY: the count / collective stream at high priority, A/B)
    cs = torch.cuda.Stream(dev, priority=CS_PRIORITY) if (world > 1 or use_cs) else None
    split_destroy = None
    if use_cs and CU_SPLIT != 0:  # the count stream on CUs of its own (A/B)
        stream, cs, split_destroy = cu_split_streams(dev, CU_SPLIT)
        sh = stream.cuda_stream
    csh = cs.cuda_stream if use_cs else None
    step_counts = [torch.zeros_like(counts), torch.zeros_like(counts)] if world > 1 else None
    k_ev = [torch.cuda.Event(), torch.cuda.Event()]
    done_ev = [torch.cuda.Event(), torch.cuda.Event()]
    pend = [False, False]
    kstep = [0]

    def step(ev=None):
        b = kstep[0] & 1
        kstep[0] += 1
        if world > 1:
            if pend[b]:
                stream.wait_event(done_ev[b])  # its previous all-reduce + add are done
            step_counts[b].zero_()
        tgt = counts if world == 1 else step_counts[b]
        if ev is not None:
            ev[0].record(stream)
        ctx.classify_dev(pk, off, ln, n, ul, w["len_hint"], out, tgt if COUNTS else None,
                         stream=sh, count_stream=csh)
        if ev is not None:
            ev[1].record(stream)
        if world > 1:
            k_ev[b].record(stream)
            cs.wait_event(k_ev[b])
            coll(step_counts[b], cs)
            with torch.cuda.stream(cs):
                counts.add_(step_counts[b])
            done_ev[b].record(cs)
            pend[b] = True

    # clock ramp (untimed, before the W warmup steps): the burst kernel runs
    # back to back for RAMP_MS of wall time without counts, so the timed steps
    # see the GPU at its loaded clocks (W = 5 alone left cfg2 7% slow: 0.279
    # vs 0.259 ms after 200 warmup steps, profiles/r01h/bench_warmup.txt)
    t_start = time.perf_counter()
    t_ramp = t_start + RAMP_MS / 1e3
    while RAMP_MS > 0 and time.perf_counter() < t_ramp:
        for _ in range(8):
            ctx.classify_dev(pk, off, ln, n, ul, w["len_hint"], out, None, stream=sh)
        torch.cuda.synchronize(dev)
    # then until steady: windows of 8 back-to-back bursts (HIP events) until a
    # window is no more than 1% faster than the best before it, at most
    # RAMP_MAX_S (a box can
    # come out of the previous process's load with the burst kernel running
    # 10% slow for seconds: profiles/r04i, r05b)
    ramp_win = []
    while RAMP_MS > 0 and time.perf_counter() - t_start < RAMP_MAX_S:
        a_ev, b_ev = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a_ev.record(stream)
        for _ in range(8):
            ctx.classify_dev(pk, off, ln, n, ul, w["len_hint"], out, None, stream=sh)
        b_ev.record(stream)
        torch.cuda.synchronize(dev)
        ramp_win.append(a_ev.elapsed_time(b_ev) / 8)
        if len(ramp_win) >= 3 and ramp_win[-1] >= 0.99 * min(ramp_win[:-1]):
            break  # no longer getting faster
    ramp_info = dict(ms=round((time.perf_counter() - t_start) * 1e3, 1), windows=len(ramp_win),
                     first_ms=round(ramp_win[0], 4) if ramp_win else None,
                     last_ms=round(ramp_win[-1], 4) if ramp_win else None)
    for _ in range(warmup):
        step()
    # kernel time: one HIP event pair on the kernel's stream around the K
    # timed steps (back-to-back launches).  Per-step event pairs cost ~3 us of
    # GPU idle each between bursts (0.2583 vs 0.2516 ms per step at cfg2, r02j)
    ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    stage(rank, f"{name}: timed steps")
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    ev[0].record(stream)
    for k in range(steps):
        step()
    if cs is not None:
        stream.wait_stream(cs)  # the last step's counts (and all-reduce) are inside the window
    ev[1].record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        torch.distributed.barrier()
    el = time.perf_counter() - t0
    kms = [ev[0].elapsed_time(ev[1]) / max(steps, 1)]
    per_rank = None
    ar_ms = None
    if world > 1:
        # the collective alone: `steps` count all-reduces back to back on the
        # collective stream (HIP events on that stream), after the timed region
        aev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        torch.distributed.barrier()
        torch.cuda.synchronize(dev)
        aev[0].record(cs)
        for _ in range(steps):
            coll(step_counts[0], cs)
        aev[1].record(cs)
        torch.cuda.synchronize(dev)
        ar_ms = aev[0].elapsed_time(aev[1]) / max(steps, 1)
        per_rank, el = gather_rank_stats(world, el, steps, kms[0], ar_ms, n)
    kdisp = kernel_dispatches(ctx, pk, off, ln, n, ul, w["len_hint"], out, counts, stream, csh,
                              dev, alg_bytes, cs if use_cs else None)
    # counts: every delivered verdict counted once per step, on every rank
    # after the all-reduce (the global histogram)
    v = out[:n * 16].view(n, 16)
    n_ok = int((v[:, 11].view(torch.int8) == 0).sum().item())
    total_steps = warmup + steps
    counted = int(counts.sum().item())
    n_ok_all = n_ok
    if world > 1:
        t = torch.tensor([n_ok], dtype=torch.int64)
        torch.distributed.all_reduce(t)
        n_ok_all = int(t.item())
    expect = n_ok_all * total_steps if COUNTS else None
    # the count vector flow by flow: (all-reduced) counts == total_steps x the
    # sum over ranks of each rank's histogram of its own delivered verdicts
    # (UDP flow k -> k, TCP flow k -> nu + k), exchanged over the control plane
    counts_match = None
    if COUNTS:
        ok = v[:, 11].view(torch.int8) == 0
        fid = v[:, 0:4].contiguous().view(torch.int32).flatten().to(torch.int64)
        cidx = torch.where(v[:, 10] == R.CLS_UDP, fid, fid + len(udp))[ok]
        hist = torch.bincount(cidx, minlength=nflows)[:nflows].cpu()
        if world > 1:
            torch.distributed.all_reduce(hist)
        counts_match = bool(torch.equal(counts.cpu(), hist * total_steps))
    kavg = float(np.mean(kms))
    n_all, alg_all = n, alg_bytes
    if world > 1:  # the whole job: frames and algorithmic bytes of every rank
        t = torch.tensor([n, alg_bytes], dtype=torch.int64)
        torch.distributed.all_reduce(t)
        n_all, alg_all = int(t[0].item()), int(t[1].item())
    res = dict(
        workload=name, desc=w["desc"], frames_per_step=n_all, frames_this_rank=n,
        nflows=nflows, mpps=n_all * steps / el / 1e6,
        gbps=alg_all * steps / el / 1e9, ms_per_step=el / steps * 1e3,
        kernel_ms_avg=kavg,
        alg_bytes_per_launch=alg_bytes, frame_bytes=frame_bytes,
        rc0_frac=n_ok / max(n, 1), counts_ok=(expect is None or counted == expect),
        counts_match=counts_match,
        setup_s=round(t_setup, 2), count_stream=bool(COUNTS and csh is not None),
        ramp=ramp_info,
        shard_mode=shard_mode if world > 1 else None,
    )
    if world > 1:
        res["allreduce_ms"] = round(ar_ms, 4)
        res["allreduce_bytes"] = 8 * nflows
        res["per_rank"] = per_rank
    achieved = alg_bytes / (kavg * 1e-3) / 1e9  # this rank's kernel (HIP events)
    res["roofline"] = dict(bound="hbm", achieved=round(achieved, 1), peak=HBM_PEAK_GBS,
                           unit="GB/s", frac=round(achieved / HBM_PEAK_GBS, 4),
                           traffic=pmc_traffic(name) if world == 1 else None,
                           kernel=kdisp)
    g = w["gen"]
    if world == 1 and g.get("frame_len") and not g.get("packed") and not g.get("size_mode") \
            and g["slot_bytes"] <= 1536:
        # the same burst read in the classify kernel's slot shape, and plainly,
        # in this process (a same-process access-shape table)
        res["slot_shape_ceiling"] = slot_ceiling(dev.index or 0, pk, n, g["slot_bytes"],
                                                 g["frame_len"], kdisp.get("median_ms"))
    # parity of this run: a seeded sample of the verdicts regenerated on the CPU
    stage(rank, f"{name}: parity")
    t_par = time.perf_counter()
    checked, bad, first_bad = parity_check(name, gcfg, udp, tcb, out, n, gidx, ul,
                                           parity_sample, seed=1000 + rank,
                                           threads=oracle_threads)
    if world > 1:
        t = torch.tensor([checked, bad], dtype=torch.int64)
        torch.distributed.all_reduce(t)
        checked, bad = int(t[0].item()), int(t[1].item())
    res["parity"] = dict(checked=checked, mismatches=bad,
                         sample="seeded uniform sample of this run's verdicts (every rank), "
                                "frames regenerated on the CPU and classified by "
                                "oracle/ref_cpu.c", seconds=round(time.perf_counter() - t_par, 2))
    if first_bad:
        log(f"PARITY FAILURE {name}: {first_bad}")
    t_dg = time.perf_counter()
    res["digest"] = burst_digest(name, out, n, gidx, counts, warmup + steps, rank, world,
                                 shard_mode)
    res["digest"]["seconds"] = round(time.perf_counter() - t_dg, 2)
    if res["digest"]["digest_ok"] is False:
        log(f"DIGEST MISMATCH {name}: {res['digest']}")
    if V8 and world == 1:
        res["verdict8"] = verdict8_leg(name, ctx, pk, off, ln, n, ul, w["len_hint"], out, nflows,
                                       steps, warmup, dev, stream, csh, frame_bytes)
    if TX and world == 1:  # K2 (TX checksum fill) over the same burst, in place
        tev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        for _ in range(warmup):
            ctx.tx_cksum_dev(pk, off, ln, n, ul, w["len_hint"], stream=sh)
        tev[0].record(stream)
        for _ in range(steps):
            ctx.tx_cksum_dev(pk, off, ln, n, ul, w["len_hint"], stream=sh)
        tev[1].record(stream)
        torch.cuda.synchronize(dev)
        tms = tev[0].elapsed_time(tev[1]) / max(steps, 1)
        tx_bytes = frame_bytes + 6 * n + 4 * n
        res["tx_cksum"] = dict(kernel_ms_avg=round(tms, 4), mpps=round(n / tms / 1e3, 1),
                               gb_per_s=round(tx_bytes / tms / 1e6, 1),
                               frac=round(tx_bytes / tms / 1e6 / HBM_PEAK_GBS, 4),
                               traffic=pmc_traffic(name, "tx_cksum"))
    if split_destroy is not None:
        split_destroy()
        res["cu_split"] = dict(count_cus=CU_SPLIT, note="count stream on CUs of its own, "
                               "classify on the rest (hipExtStreamCreateWithCUMask)")
    del pk, off, ln, out
    torch.cuda.empty_cache()
    return res


KDISP = 20  # dispatches of the per-dispatch pass (roofline.kernel)


def kernel_dispatches(ctx, pk, off, ln, n, ul, len_hint, out, counts, stream, csh, dev, alg_bytes,
                      cs=None):
    """roofline.kernel: the dominant kernel dispatch by dispatch, so that a
    kernel trace of the same run (rocprofv3 --kernel-trace) can confirm it.
    KDISP untimed classify dispatches after the timed steps, each between its
    own HIP event pair on the kernel's stream, counts on (into a scratch
    vector: the run's counts stay exact).  Where the counts are separate passes
    on the count stream cs, each dispatch first waits for the previous one's
    passes, so that no slab pass shares the GPU with the dispatch being timed
    (in the steps they overlap the next classify; a kernel trace times each
    kernel on its own).  A dispatch measured alone includes its ramp-up and
    drain, which back-to-back steps overlap with the next dispatch."""
    name, variant = ctx.kernel_variant(len_hint)
    scratch = torch.zeros_like(counts) if COUNTS else None
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(KDISP)]
    torch.cuda.synchronize(dev)
    for a, b in evs:
        if cs is not None:
            stream.wait_stream(cs)
        a.record(stream)
        ctx.classify_dev(pk, off, ln, n, ul, len_hint, out, scratch, stream=stream.cuda_stream,
                         count_stream=csh)
        b.record(stream)
    torch.cuda.synchronize(dev)
    t = sorted(a.elapsed_time(b) for a, b in evs)
    mean = float(np.mean(t))
    med = t[len(t) // 2]
    del scratch
    return dict(name=name, variant=variant, dispatches=KDISP, mean_ms=round(mean, 4),
                median_ms=round(med, 4), min_ms=round(t[0], 4), max_ms=round(t[-1], 4),
                achieved=round(alg_bytes / (med * 1e-3) / 1e9, 1),
                frac=round(alg_bytes / (med * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                timing="per dispatch: one HIP event pair each on the kernel's stream, "
                       "untimed pass after the steps; achieved and frac from median_ms")


def verdict8_leg(name, ctx, pk, off, ln, n, ul, len_hint, out16, nflows, steps, warmup, dev,
                 stream, csh, frame_bytes):
    """the same steps writing compact 8-B verdicts (rxg_classify_dev8): time,
    rate, and every verdict against the projection of this run's 16-B
    verdicts (pinned by the digests above) and the golden verdict8_sha256"""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import digest as D  # parity leg only
    sh = stream.cuda_stream
    out8 = torch.empty(max(n, 1) * 8, dtype=torch.uint8, device=dev)
    cnt = torch.zeros(max(nflows, 1), dtype=torch.int64, device=dev) if COUNTS else None
    for _ in range(warmup):
        ctx.classify_dev8(pk, off, ln, n, ul, len_hint, out8, cnt, stream=sh, count_stream=csh)
    ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    torch.cuda.synchronize(dev)
    ev[0].record(stream)
    for _ in range(steps):
        ctx.classify_dev8(pk, off, ln, n, ul, len_hint, out8, cnt, stream=sh, count_stream=csh)
    if csh is not None:
        stream.wait_stream(torch.cuda.ExternalStream(csh, device=dev))
    ev[1].record(stream)
    torch.cuda.synchronize(dev)
    ms = ev[0].elapsed_time(ev[1]) / max(steps, 1)
    same = bool(torch.equal(out8[:n * 8], D.verdict8_torch(out16[:n * 16])))
    sha = D.sha256_bytes(out8[:n * 8].cpu().numpy())
    try:
        gold = D.load_golden().get(name, {}).get("verdict8_sha256")
    except OSError:
        gold = None
    alg = frame_bytes + 14 * n
    r = dict(ms_per_step=round(ms, 4), mpps=round(n / ms / 1e3, 1),
             alg_bytes_per_launch=alg, gb_per_s=round(alg / ms / 1e6, 1),
             frac=round(alg / ms / 1e6 / HBM_PEAK_GBS, 4), equals_projection=same,
             verdict8_sha256=sha, digest_ok=(sha == gold) if gold else None)
    del out8, cnt
    return r


def burst_digest(name, out, n, gidx, counts, total_steps, rank, world, shard_mode="direct"):
    """the whole burst against tests/golden/digests.json (the oracle's verdicts
    of every frame of the workload's burst, computed offline by
    tests/golden/make_digests.py): N = 1, the SHA-256 of all n x 16 verdict
    bytes, the order-free frame digest and the per-flow histogram (the
    counts after the run / the bursts counted); N > 1, the frame digest of the
    golden burst's frames (global index < n) summed over the ranks that hold
    them."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import digest as D  # parity leg only
    try:
        gold = D.load_golden().get(name)
    except OSError:
        gold = None
    dev = out.device
    v = out[:n * 16]
    if world > 1 and shard_mode == "direct":
        # each rank's frames are its own shard stream, not frames of the
        # golden burst: the per-rank oracle sample and the count check
        # (counts_match) are the parity evidence at N > 1
        return dict(golden=False, digest_ok=None,
                    scope="N > 1, shards generated per rank: no golden burst; see parity "
                          "(oracle sample per rank) and counts_match")
    r = dict(golden=gold is not None)
    if world == 1:
        idx = torch.arange(n, dtype=torch.int64, device=dev)
        r["frames"] = n
        r["frame_digest"] = f"{D.frame_digest_torch(idx, v):016x}"
        r["verdict_sha256"] = D.sha256_bytes(v.cpu().numpy())
        c = counts.cpu().numpy().view(np.uint64)
        whole = bool(np.all(c % np.uint64(total_steps) == 0))
        r["counts_sha256"] = D.counts_sha256(c // np.uint64(total_steps)) if whole else None
        if gold is not None:
            r["digest_ok"] = (n == gold["frames"] and r["verdict_sha256"] == gold["verdict_sha256"]
                              and r["frame_digest"] == gold["frame_digest"]
                              and (not COUNTS or r["counts_sha256"] == gold["counts_sha256"]))
    else:
        g = torch.from_numpy(gidx).to(dev)
        lim = gold["frames"] if gold is not None else rxdist.WORKLOADS[name]["n"]
        keep = torch.nonzero(g < lim).flatten()
        part = D.frame_digest_torch(g.index_select(0, keep),
                                    v.view(n, 16).index_select(0, keep)) if len(keep) else 0
        t = torch.tensor([part - (1 << 64) if part >= 1 << 63 else part, len(keep)],
                         dtype=torch.int64)
        allr = [torch.zeros_like(t) for _ in range(world)]
        torch.distributed.all_gather(allr, t)
        tot = sum(int(x[0]) for x in allr) & D._M64
        r["frames"] = sum(int(x[1]) for x in allr)
        r["frame_digest"] = f"{tot:016x}"
        r["scope"] = "frames 0..n-1 of the global burst (the golden burst), over all ranks"
        if gold is not None:
            r["digest_ok"] = (r["frames"] == gold["frames"]
                              and r["frame_digest"] == gold["frame_digest"])
    r.setdefault("digest_ok", None)  # None: no golden entry for this workload
    return r


def lib_sha256():
    import hashlib
    h = hashlib.sha256()
    with open(R.LIB_PATH, "rb") as f:
        for b in iter(lambda: f.read(1 << 20), b""):
            h.update(b)
    return h.hexdigest()


def pmc_traffic(name, kernel=None):
    """HBM bytes per launch from the newest committed PMC summary for this
    workload (profiles/pmc_*.json, written by tools/pmc_traffic.py) — only if
    that summary was measured on THIS librxgpu.so (same SHA-256), else None:
    a kernel edit without a fresh PMC pass publishes no stale traffic.
    kernel=None: K1 (rx_classify); "tx_cksum": K2."""
    sha = lib_sha256()
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc_*.json")))
    for f in reversed(files):
        try:
            d = json.load(open(f))
        except Exception:
            continue
        if d.get("librxgpu_sha256") != sha or d.get("variant"):
            continue  # another library build, or a forced (tuning) kernel variant
        w = d.get("workloads", {}).get(name)
        if w is not None:
            if kernel is not None:
                w = w.get(kernel)
                if w is None:
                    continue
            return w.get("hbm_bytes_per_launch")
    return None


# ---------------------------------------------------------------------------
# Oracle legs (test infrastructure: the checker, and the CPU baseline)
def _oracle():
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_bind as O  # parity + cpu_baseline legs only
    return O


_TABLES = {}


def oracle_tables(name, udp, tcb, opt="O2"):
    """the reference's head-inserted lists, built once per workload and build"""
    O = _oracle()
    key = (name, opt)
    if key not in _TABLES:
        _TABLES[key] = O.Tables(udp, tcb, which=O.lib if opt == "O2" else O.lib_O0())
    return _TABLES[key]


def regen(cfg, gidx, ul):
    """frames gidx[k] of a workload's burst, regenerated on the CPU (the
    pktgen is a pure function of (cfg, i)), one slot_bytes slot each"""
    slot = cfg.slot_bytes
    buf = np.zeros(len(gidx) * slot + 64, np.uint8)
    lens = np.zeros(len(gidx), np.uint16)
    for j, i in enumerate(gidx):
        p, _, l = R.gen_host(cfg, int(i), 1, ul)
        buf[j * slot:j * slot + slot] = p[:slot]
        lens[j] = l[0]
    offs = (np.arange(len(gidx), dtype=np.uint64) * slot >> ul).astype(np.uint32)
    return buf, offs, lens


def _threaded(fn, parts, threads):
    """run fn(part) over parts on `threads` host threads (ctypes drops the GIL)"""
    import concurrent.futures as cf
    if threads <= 1 or len(parts) <= 1:
        return [fn(p) for p in parts]
    with cf.ThreadPoolExecutor(threads) as ex:
        return list(ex.map(fn, parts))


def parity_check(name, cfg, udp, tcb, out, n, gidx, ul, sample, seed, threads=1):
    """bit-exact check of a seeded sample of this run's verdicts against the
    oracle on the same frames; returns (checked, mismatches, first mismatch)"""
    if sample <= 0 or n == 0:
        return 0, 0, None
    rng = np.random.default_rng(seed)
    loc = np.arange(n) if sample >= n else np.sort(rng.choice(n, sample, replace=False))
    sel = torch.from_numpy(loc.astype(np.int64)).to(out.device)
    got = out[:n * 16].view(n, 16).index_select(0, sel).cpu().numpy().reshape(-1)
    got = got.view(R.VERDICT_DTYPE)
    g = loc if gidx is None else gidx[loc]
    buf, offs, lens = regen(cfg, g, ul)
    tb = oracle_tables(name, udp, tcb)
    parts = np.array_split(np.arange(len(g)), max(1, min(threads, len(g) // 64 or 1)))
    want = np.concatenate(_threaded(lambda ix: tb.classify(buf, offs[ix], lens[ix], ul), parts,
                                    threads))
    bad = np.nonzero(np.any(got.view(np.uint8).reshape(-1, 16) !=
                            want.view(np.uint8).reshape(-1, 16), axis=1))[0]
    first = None
    if len(bad):
        k = int(bad[0])
        first = dict(frame=int(g[k]), got=str(got[k]), want=str(want[k]))
    return len(g), int(len(bad)), first


def host_cores():
    """the host CPU as the bench sees it: nproc, the affinity mask, the cgroup
    quota, the thread budget (OMP_NUM_THREADS: the GPU box's CPU share per
    GPU) and the model"""
    nproc = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = nproc
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        pass
    use = aff if quota is None else max(1, min(aff, int(quota)))
    share = os.environ.get("OMP_NUM_THREADS")
    if share and share.isdigit():
        use = max(1, min(use, int(share)))
    model = platform.processor() or platform.machine()
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return dict(nproc=nproc, affinity=aff, cgroup_quota=quota, threads=use, model=model)


CPU_SAMPLE = {"cfg1": 100000, "cfg2": 1 << 20, "cfg3": 1 << 16, "cfg4": 1 << 16,
              "cfg5": 1 << 14}


def cpu_rate(tb, pk, off, ln, ul, budget_s, threads=1):
    """frames/s of the oracle over the sample, cycled until ~budget_s of
    work per thread; threads > 1: the sample RSS-split over the threads (the
    same 5-tuple sharding as the GPUs, rxg_rss_split), one shard per thread"""
    k = min(len(off), 256)  # calibrate (the list scans cost ~3 ms per lookup at 1M tcbs)
    t0 = time.perf_counter()
    tb.classify(pk, off[:k], ln[:k], ul)
    per = (time.perf_counter() - t0) / k
    target = max(1, int(budget_s / max(per, 1e-9)))  # frames per thread
    if threads <= 1:
        shards = [np.arange(len(off))]
    else:
        # RSS shards (at most RXG_MAX_SHARDS = 64 queues), each cut into
        # contiguous pieces when there are more threads than queues
        nq = min(threads, 64)
        first, perm = R.rss_split(pk, off, ln, ul, nq)
        per = -(-threads // nq)
        shards = [piece for s in range(nq)
                  for piece in np.array_split(perm[first[s]:first[s + 1]], per)]
        shards = [s for s in shards if len(s)]

    def work(ix):
        o, l = np.ascontiguousarray(off[ix]), np.ascontiguousarray(ln[ix])
        # at least 16 frames of the thread's shard: a lookup's cost depends on
        # where its flow sits in the list, so one or two frames per thread (1M
        # tcbs, nproc threads) are not a sample
        want = max(target, min(len(ix), 16))
        done = 0
        while done < want:
            m = min(len(ix), want - done)
            tb.classify(pk, o[:m], l[:m], ul)
            done += m
        return done
    t0 = time.perf_counter()
    done = _threaded(work, shards, threads)
    el = time.perf_counter() - t0
    return sum(done) / el, sum(done), el


def cpu_baseline(name, budget_s, cores):
    """SURVEY.md §8(d) / BASELINE.md §3: the oracle (the reference algorithm:
    list-scan lookups, per-word checksum; printf disabled) at -O2 and at -O0
    (the reference's own build flags), on 1 core (the reference's single
    pkt_process lcore, netfamily.c:427) and on every usable host core with
    the sample RSS-sharded; a bounded, cycled sample of the same workload."""
    w = rxdist.WORKLOADS[name]
    cfg = rxdist.gen_cfg(name)
    ul = w["unit_log2"]
    sample = min(CPU_SAMPLE[name], w["n"])
    pk, off, ln = R.gen_host(cfg, 0, sample, ul)
    udp, tcb = R.gen_flows(cfg)
    res = {}
    for opt in ("O2", "O0"):
        tb = oracle_tables(name, udp, tcb, opt)
        r1, d1, e1 = cpu_rate(tb, pk, off, ln, ul, budget_s)
        rn, dn, en = cpu_rate(tb, pk, off, ln, ul, budget_s / 2, cores["threads"])
        # every logical CPU the host reports (nproc threads), whatever the
        # cgroup quota allows this process: the quota, not the thread count,
        # then bounds the rate (reported beside it)
        # (per-thread work scaled so the leg's total CPU time stays ~budget_s / 8
        # of the box's share: nproc threads time-share the quota)
        rp, dp, ep = cpu_rate(tb, pk, off, ln, ul,
                              budget_s / 8 * cores["threads"] / max(cores["nproc"], 1),
                              cores["nproc"])
        res[opt] = dict(one_core=dict(mpps=round(r1 / 1e6, 4), frames=d1, seconds=round(e1, 2)),
                        all_cores=dict(mpps=round(rn / 1e6, 4), frames=dn, seconds=round(en, 2),
                                       threads=cores["threads"]),
                        nproc=dict(mpps=round(rp / 1e6, 4), frames=dp, seconds=round(ep, 2),
                                   threads=cores["nproc"], cgroup_quota=cores["cgroup_quota"]))
    sampled = "sampled: " if name in ("cfg4", "cfg5") else ""
    return dict(
        value=res["O2"]["one_core"]["mpps"], unit="Mpps", cores=1, kind="port",
        sample=f"{sampled}{sample} distinct frames of {name} ({w['desc']}), cycled to the time "
               f"budget; oracle/ref_cpu.c (list-scan lookups, printf off); value = -O2 on 1 "
               f"core; all_cores = {cores['threads']} threads over an RSS split of the sample "
               f"(host: {cores['model']}, nproc {cores['nproc']}, affinity {cores['affinity']}, "
               f"cgroup quota {cores['cgroup_quota']}, threads capped at the box's CPU share; "
               f"nproc = {cores['nproc']} threads, bounded by the same cgroup quota)",
        sample_short=f"{sampled}{sample} frames of {name} cycled ~{budget_s:g} s through "
                     f"oracle/ref_cpu.c (-O2, list-scan lookups, printf off) on 1 core; "
                     f"all_cores = {cores['threads']} threads over an RSS split",
        O2=res["O2"], O0=res["O0"], host=cores)


def run_cfg1(local, dev, steps, warmup, budget_s, cores):
    """BASELINE configs[0]: 100K x 64 B UDP from a pcap, one flow.  The frames
    go through a pcap file (rxg_pcap_write / rxg_pcap_read_burst), then through
    the host-buffer path (rxg_classify_span: PCIe both ways) with every verdict
    checked against the oracle, then device-resident (rxg_classify_dev); the
    oracle times the same pcap burst at -O2 and -O0 on 1 core."""
    import tempfile
    w = rxdist.WORKLOADS["cfg1"]
    cfg = rxdist.gen_cfg("cfg1")
    n, ul = w["n"], w["unit_log2"]
    hp, ho, hl = R.gen_host(cfg, 0, n, ul)
    path = os.path.join(tempfile.gettempdir(), f"rxg_cfg1_{os.getpid()}.pcap")
    R.pcap_write(path, hp, ho, hl, ul)
    pc = R.Pcap(path)
    buf = torch.zeros(n * 64 + 64, dtype=torch.uint8).pin_memory()
    poff = torch.zeros(n, dtype=torch.int32).pin_memory()
    pln = torch.zeros(n, dtype=torch.int16).pin_memory()
    got_n, span = pc.read_burst_into(buf.numpy(), poff.numpy().view(np.uint32),
                                     pln.numpy().view(np.uint16), ul)
    pc.close()
    os.unlink(path)
    assert got_n == n, (got_n, n)
    udp, tcb = R.gen_flows(cfg)
    out = torch.zeros(n * 16, dtype=torch.uint8).pin_memory()
    ctx = R.Context(local, max_pkts=n, max_bytes=span + 64)
    ctx.flows_sync(udp, tcb)
    args = (buf.data_ptr(), span, poff.data_ptr(), pln.data_ptr(), n, ul, out.data_ptr())
    ctx.classify_span(*args)
    got = out.numpy().view(R.VERDICT_DTYPE).copy()
    bufn, offn, lnn = buf.numpy(), poff.numpy().view(np.uint32), pln.numpy().view(np.uint16)
    want = oracle_tables("cfg1", udp, tcb).classify(bufn, offn, lnn, ul)
    bad = int(np.any(got.view(np.uint8).reshape(-1, 16) != want.view(np.uint8).reshape(-1, 16),
                     axis=1).sum())
    for _ in range(3):
        ctx.classify_span(*args)
    t0 = time.perf_counter()
    for _ in range(steps):
        ctx.classify_span(*args)
    e2e_ms = (time.perf_counter() - t0) / steps * 1e3
    # device-resident: the same burst in HBM
    d_pk, d_off, d_ln = buf.to(dev), poff.to(dev), pln.to(dev)
    d_out = torch.empty(n * 16, dtype=torch.uint8, device=dev)
    sh = torch.cuda.current_stream(dev).cuda_stream
    for _ in range(warmup + 20):
        ctx.classify_dev(d_pk, d_off, d_ln, n, ul, 64, d_out, None, stream=sh)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(steps):
        ctx.classify_dev(d_pk, d_off, d_ln, n, ul, 64, d_out, None, stream=sh)
    b.record()
    torch.cuda.synchronize(dev)
    dev_ms = a.elapsed_time(b) / steps
    dev_bad = int((d_out.cpu().numpy().view(R.VERDICT_DTYPE).tobytes() != want.tobytes()))
    ctx.close()
    res = dict(workload="cfg1", desc=w["desc"], frames=n,
               parity=dict(checked=n, mismatches=bad, device_path_equal=(dev_bad == 0),
                           sample="every frame of the pcap burst vs oracle/ref_cpu.c"),
               rc0_frac=round(float((got["rc"] == 0).mean()), 4),
               pcie_inclusive=dict(ms_per_burst=round(e2e_ms, 4), mpps=round(n / e2e_ms / 1e3, 2)),
               device_resident=dict(ms_per_burst=round(dev_ms, 5), mpps=round(n / dev_ms / 1e3, 1)))
    if budget_s > 0:
        cpu = {}
        for opt in ("O2", "O0"):
            tb = oracle_tables("cfg1", udp, tcb, opt)
            r1, d1, e1 = cpu_rate(tb, bufn, offn, lnn, ul, budget_s)
            cpu[opt] = dict(mpps=round(r1 / 1e6, 4), frames=d1, seconds=round(e1, 2))
        res["cpu_baseline"] = dict(
            value=cpu["O2"]["mpps"], unit="Mpps", cores=1, kind="port",
            sample=f"the same pcap burst ({n} frames), cycled; oracle/ref_cpu.c front end "
                   f"(udp.c:11-19 lookup + verdict), 1 thread; host {cores['model']}",
            O2=cpu["O2"], O0=cpu["O0"])
    return res


SOCK_CASES = {
    # BASELINE configs[1]: 1024 UDP sockets bound to :20000-21023, 64-B datagrams
    "cfg2": dict(burst=32768, bursts=30),
    # BASELINE configs[2]: 4096 connections to the listener on :9999 (each
    # established by a SYN / ACK exchange through the stack), 1500-B segments
    "cfg3": dict(burst=16384, bursts=20),
}


def gpu_local_cpus(local):
    """the CPUs this process may use on the GPU's NUMA node (sysfs), else all
    of them: (cpus, node)"""
    aff = sorted(os.sched_getaffinity(0))
    try:
        p = torch.cuda.get_device_properties(local)
        bdf = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
        with open(f"/sys/bus/pci/devices/{bdf}/numa_node") as f:
            node = int(f.read())
        if node >= 0:
            with open(f"/sys/devices/system/node/node{node}/cpulist") as f:
                cl = f.read().strip()
            on = set()
            for part in cl.split(","):
                a, _, b = part.partition("-")
                on.update(range(int(a), int(b or a) + 1))
            loc = [c for c in aff if c in on]
            if len(loc) >= 2:
                return loc, node
    except (OSError, ValueError, AttributeError, RuntimeError):
        pass
    return aff, None


def socket_api(local, name, budget_s, cores, with_cpu=True):
    """The kept socket API's rate: bursts through
    nstack_rx_burst — GPU classify (rxg_process_mbufs: staging, PCIe, K1) then
    host delivery into the sockets' receive rings with the reference's
    offload / tcp_fragment semantics (udp.c:25-52, tcp.c:133-185) — and the
    application reading every socket (nrecvfrom / nrecv, common.c:462-565).
    CPU baseline: oracle/ref_stack.c, the reference's per-frame
    udp_process / tcp_process and socket calls, over the same frames."""
    w = rxdist.WORKLOADS[name]
    cfg = rxdist.gen_cfg(name)
    ul = w["unit_log2"]
    sc = SOCK_CASES[name]
    B, K = sc["burst"], sc["bursts"]
    udp, tcb = R.gen_flows(cfg)
    L = "192.168.100.77"
    ns = R.NStack(local, max_burst=B, max_bytes=B * cfg.slot_bytes + 4096)
    res = dict(workload=name, frames_per_burst=B)
    # the protocol thread (this one) and the application thread on two
    # neighbouring cores of the GPU's NUMA node, as a DPDK application pins
    # its lcores (EAL -l): threads left to migrate across the two sockets of
    # the box paid remote cache-line transfers on every socket ring
    lcpus, node = gpu_local_cpus(local)
    pair = (lcpus[0], lcpus[1]) if len(lcpus) >= 2 else None
    res["lcores"] = dict(cpus=list(pair) if pair else None, numa_node=node)
    old_aff = os.sched_getaffinity(0)
    if pair:
        os.sched_setaffinity(0, {pair[0]})
    try:
        setup = []  # (frames for the handshake), applied to both stacks
        if name == "cfg2":
            # the reference's descriptor table (common.h:33, fds 3-1023) holds
            # 1,021 sockets: the last 3 of the 1,024 ports stay unbound, and
            # their frames miss (rc -3), as they would in the reference
            bound = 0
            for u in udp:
                fd = ns.socket(R.SOCK_DGRAM)
                if fd >= 0 and ns.bind(fd, L, int.from_bytes(int(u["localport"]).to_bytes(2, "little"),
                                                              "big")) == 0:
                    bound += 1
            res["sockets_bound"] = bound
        else:
            sys.path.insert(0, os.path.join(ROOT, "tests"))
            import frames as F  # test infrastructure: the handshake frames
            lfd = ns.socket(R.SOCK_STREAM)
            ns.bind(lfd, L, 9999)
            ns.listen(lfd)
            for t in tcb[1:]:
                sip = ".".join(str(b) for b in int(t["sip"]).to_bytes(4, "little"))
                sp = int.from_bytes(int(t["sport"]).to_bytes(2, "little"), "big")
                setup.append((F.tcp_frame(sip, sp, L, 9999, b"", flags=0x02, seq=1),
                              F.tcp_frame(sip, sp, L, 9999, b"", flags=0x10, seq=2)))
            for k in (0, 1):
                for j in range(0, len(setup), 4096):
                    fr = [s[k] for s in setup[j:j + 4096]]
                    ns.rx_burst(fr)
            res["established"] = int(ns.tcb_count()) - 1
        pk, off, ln = R.gen_host(cfg, 0, B, ul)
        # the mbuf pool: NSET bursts' worth of frames in distinct memory (the
        # same bytes in each), registered with the stack once, as a DPDK
        # application registers its mempool (rte_mempool_mem_iter): the GPU
        # pulls each burst's frames over PCIe instead of a host gather + copy.
        # In place (nstack_set_rx_inplace, the A/B here), a connection's
        # receive fragments point into these frames and hold their mbufs
        # (refcnt) until the application has read them, so a set is reused
        # only once every one of its counts is back to 0 (the NIC refilling
        # its ring from free mbufs).  The default is the pooled payload
        # buffers: measured faster at cfg3 in every arrangement (r06d:
        # sequential 6.51 vs 5.81 Mpps, two threads 8.62 vs 7.45, pipelined
        # two threads 10.73 vs 6.80)
        NSET = 4
        span = len(pk)
        pool = np.empty(NSET * span, np.uint8)
        sets = []
        for j in range(NSET):
            seg = pool[j * span:(j + 1) * span]
            seg[:] = pk
            a_j, k_j = R.NStack.mbufs_over(seg, off, ln, ul)
            rc_j = np.frombuffer(k_j, np.uint8).reshape(B, 128)[:, 18:20].view(np.uint16)
            rc_j[:] = 0  # the pool keeps no reference of its own: free at count 0
            sets.append((a_j, k_j, rc_j))
        try:
            ns.register_host(pool.ctypes.data, pool.nbytes)
            res["pool_registered"] = True
        except R.RxgError as e:  # reported, and the host gather carries the bursts
            res["pool_registered"] = repr(e)
        ns.set_rx_inplace(False)
        res["tcp_inplace"] = False
        kset = [0]
        pool_waits = [0]

        def next_set():
            """the next mbuf set whose frames no fragment holds any more"""
            a_j, _, rc_j = sets[kset[0] % NSET]
            kset[0] += 1
            if rc_j.any():
                pool_waits[0] += 1
                t_end = time.perf_counter() + 5.0
                while rc_j.any():
                    if time.perf_counter() > t_end:
                        raise RuntimeError("mbuf set still held after 5 s")
                    time.sleep(0)
                    ns.reclaim()  # (what the application thread has read lets go of its frames)
            return a_j
        rbuf = np.zeros(65536, np.uint8)
        ns.rx_burst_mbufs(next_set(), B)  # warm (staging, tables committed)
        ns.drain_all(rbuf)
        t_rx = t_dr = 0.0
        items = nbytes = delivered = 0
        phases = []
        for _ in range(K):
            arr = next_set()
            t0 = time.perf_counter()
            delivered += ns.rx_burst_mbufs(arr, B)
            t1 = time.perf_counter()
            phases.append(ns.last_burst_phases())
            g, nb = ns.drain_all(rbuf)
            t2 = time.perf_counter()
            t_rx += t1 - t0
            t_dr += t2 - t1
            items += g
            nbytes += nb
        # where rx_burst's time goes (nstack_last_burst_phases: host gather,
        # then copy in / K1 / K3 + K4 / copy out from HIP events, then the host
        # delivery steps), median over the bursts
        res["rx_burst_phases_ms"] = {k: round(float(np.median([p[k] for p in phases])), 4)
                                     for k in phases[0]}
        def ab_run(pipelined=False):  # the sequential loop again, for an A/B
            h_rx = h_dr = 0.0
            h_items = 0
            h_ph = []
            if pipelined:  # burst k+1 on the GPU while burst k is delivered and read
                ns.rx_submit_mbufs(next_set(), B)
            for k in range(K):
                t0 = time.perf_counter()
                if pipelined:
                    if k + 1 < K:
                        ns.rx_submit_mbufs(next_set(), B)
                    ns.rx_complete_mbufs()
                else:
                    ns.rx_burst_mbufs(next_set(), B)
                t1 = time.perf_counter()
                h_ph.append(ns.last_burst_phases())
                g, _ = ns.drain_all(rbuf)
                h_rx += t1 - t0
                h_dr += time.perf_counter() - t1
                h_items += g
            return dict(mpps=round(B * K / (h_rx + h_dr) / 1e6, 3),
                        rx_burst_ms=round(h_rx / K * 1e3, 3), app_recv_ms=round(h_dr / K * 1e3, 3),
                        received_equal=h_items == items,
                        rx_burst_phases_ms={k: round(float(np.median([p[k] for p in h_ph])), 4)
                                            for k in h_ph[0]})
        # A/B: in place (the round-5 default): no payload gathered or copied
        # back; the fragments point into the frames and hold their mbufs
        ns.set_rx_inplace(True)
        res["inplace"] = ab_run()
        ns.set_rx_inplace(False)
        # A/B: pipelined (nstack_rx_submit / nstack_rx_complete): burst k+1
        # crosses PCIe and goes through the kernels while burst k is delivered
        # and read (the first submit is outside the clock, as a loop's first
        # burst would be in flight already)
        res["pipelined"] = ab_run(pipelined=True)
        ns.set_rx_inplace(True)
        res["inplace_pipelined"] = ab_run(pipelined=True)
        ns.set_rx_inplace(False)
        # A/B: each burst as two halves, both on the GPU at once
        # (nstack_set_halves; off by default)
        ns.set_halves(B // 2)
        res["halves"] = ab_run()
        ns.set_halves(0)
        # A/B: the registered pool pulled by the device frame by frame instead
        # of copied as one span (rxg_tune_ingest)
        if res.get("pool_registered") is True:
            ns.tune_ingest(R.INGEST_PULL)
            res["ingest_pull"] = ab_run()
            ns.tune_ingest(R.INGEST_AUTO)
        # the same bursts with the application on its own thread, as the
        # reference runs it (app lcore beside the protocol lcore,
        # netfamily.c:424-430): the app drains every socket in a loop while the
        # protocol thread runs the bursts (nstack_rx_burst releases the stack's
        # lock while a burst is on the GPU)
        import threading

        # the application lcore in C (tools/libappthread.so: nstack_drain_all
        # in a loop, waiting on the deliveries counter when a pass finds
        # nothing); a Python thread in that role measured the interpreter's
        # lock hand-offs, not the stack
        applib = _appthread_lib()

        def overlapped(cpus=None, unpin=False, pipelined=False):
            main_aff = os.sched_getaffinity(0)
            if cpus:
                os.sched_setaffinity(0, {cpus[0]})
            elif unpin:
                os.sched_setaffinity(0, old_aff)
            d0, s0, c0 = int(ns.stat(1)), int(ns.stat(5)), int(ns.stat(6))
            w0 = [int(ns.stat(8 + j)) for j in range(3)]
            pw0 = int(ns.stat(11))
            ov_rx, ov_ph, ov_cp, ov_tr = [], [], [], []
            w_pool0 = pool_waits[0]
            r = AppResult()
            t0 = time.perf_counter()
            if applib.app_start(cpus[1] if cpus else -1, 0) != 0:
                raise RuntimeError("app_start failed")
            try:
                if pipelined:
                    ns.rx_submit_mbufs(next_set(), B)
                for k in range(K):
                    a0 = time.perf_counter()
                    if pipelined:
                        if k + 1 < K:
                            ns.rx_submit_mbufs(next_set(), B)
                        ns.rx_complete_mbufs()
                    else:
                        ns.rx_burst_mbufs(next_set(), B)
                    ov_rx.append(time.perf_counter() - a0)
                    ov_ph.append(ns.last_burst_phases())
                    ov_cp.append(int(ns.stat(6)))
                    ov_tr.append(int(ns.stat(7)))
            finally:
                applib.app_stop(C.byref(r))
                os.sched_setaffinity(0, main_aff)
            t_ov = time.perf_counter() - t0
            if r.err:
                raise R.RxgError(int(r.err), "nstack_drain_all (application thread)")
            return dict(mpps=round(B * K / t_ov / 1e6, 3), ms_per_burst=round(t_ov / K * 1e3, 3),
                        received=int(r.items), payload_bytes=int(r.bytes),
                        received_equal=int(r.items) == items, dropped=int(ns.stat(1)) - d0,
                        stale_bursts=int(ns.stat(5)) - s0,
                        copied_payload_bytes=int(ns.stat(6)) - c0,
                        bursts_waited_for_buffer=int(ns.stat(11)) - pw0,
                        bursts_waited_for_mbufs=pool_waits[0] - w_pool0,
                        copied_mb_by_burst=[round((b - a) / 1e6, 1) for a, b in zip([c0] + ov_cp, ov_cp)],
                        held_batches_by_burst=ov_tr,
                        app_ms_per_burst={k: round((int(ns.stat(8 + j)) - w0[j]) / 1e6 / K, 3) for j, k in
                                          enumerate(("lock_wait", "yield", "read_out"))},
                        rx_burst_ms=round(float(np.median(ov_rx)) * 1e3, 3),
                        rx_burst_mean_ms=round(float(np.mean(ov_rx)) * 1e3, 3),
                        rx_burst_phases_ms={k: round(float(np.median([p[k] for p in ov_ph])), 4)
                                            for k in ov_ph[0]},
                        app_drain_ms=round(r.drain_ms / K, 3), app_passes=int(r.passes),
                        app_empty_passes=int(r.empty), app_sleeps=int(r.sleeps),
                        app_thread="C (tools/libappthread.so)",
                        cpus=list(cpus) if cpus else None,
                        note="application thread draining while the protocol thread runs "
                             "the bursts" + ("; the two threads on the lcores above" if cpus else
                                             "; threads not pinned")
                             + ("; pipelined: burst k+1 submitted before burst k is delivered "
                                "(nstack_rx_submit / nstack_rx_complete)" if pipelined else ""))
        res["overlapped"] = overlapped(pair)
        res["overlapped_pipelined"] = overlapped(pair, pipelined=True)
        # the in-place vs pooled-payload A/B in the two-thread forms too
        ns.set_rx_inplace(True)
        res["overlapped_inplace"] = overlapped(pair)
        res["overlapped_pipelined_inplace"] = overlapped(pair, pipelined=True)
        ns.set_rx_inplace(False)
        res["overlapped_unpinned"] = overlapped(None, unpin=True)
        frame_bytes = int(ln.astype(np.int64).sum())
        res.update(bursts=K, mpps=round(B * K / (t_rx + t_dr) / 1e6, 3),
                   rx_burst_ms=round(t_rx / K * 1e3, 3), app_recv_ms=round(t_dr / K * 1e3, 3),
                   rx_burst_mpps=round(B * K / t_rx / 1e6, 3),
                   payload_gb_per_s=round(nbytes / (t_rx + t_dr) / 1e9, 3),
                   frame_gb_per_s=round(frame_bytes * K / (t_rx + t_dr) / 1e9, 3),
                   received_per_burst=items // K, udp_delivered_per_burst=delivered // K,
                   dropped=int(ns.stat(1)))
    finally:
        ns.fini()
        os.sched_setaffinity(0, old_aff)
    if with_cpu:  # the reference's path on one core: oracle/ref_stack.c
        O = _oracle()
        st = O.Stack()
        if name == "cfg2":
            for u in udp:
                fd = st.socket(2)
                st.bind(fd, int(u["localip"]), int(u["localport"]))
        else:
            fd = st.socket(1)
            st.bind(fd, R.ip_raw(L), R.port_raw(9999))
            st.listen(fd)
            for k in (0, 1):
                for s in setup:
                    st.rx(s[k])
        rbuf = np.zeros(65536, np.uint8)
        done = 0
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < budget_s:
            st.rx_burst(pk, off, ln, ul)
            st.drain_all(rbuf)
            done += B
        el = time.perf_counter() - t0
        res["cpu_baseline"] = dict(mpps=round(done / el / 1e6, 3), unit="Mpps", cores=1,
                                   kind="port", frames=done, seconds=round(el, 2),
                                   sample=f"the same {B}-frame burst, cycled: oracle/ref_stack.c "
                                          f"oracle_rx per frame + every socket read; host "
                                          f"{cores['model']}")
        res["vs_cpu"] = round(res["mpps"] / max(res["cpu_baseline"]["mpps"], 1e-9), 2)
    del sets, pool
    return res


class AppResult(C.Structure):
    """tools/appthread.c app_result"""
    _fields_ = [("items", C.c_int64), ("bytes", C.c_uint64), ("sum", C.c_uint64),
                ("passes", C.c_uint64), ("empty", C.c_uint64), ("drain_ms", C.c_double),
                ("err", C.c_int64), ("sleeps", C.c_uint64)]


def _appthread_lib():
    """tools/libappthread.so (built by __graft_entry__.build / make -C tools),
    loaded after libnstack.so so that it binds the same stack"""
    p = os.path.join(ROOT, "tools", "libappthread.so")
    if not os.path.exists(p):
        raise RuntimeError(f"{p} missing: run make -C tools")
    lib = C.CDLL(p)
    lib.app_start.argtypes = [C.c_int, C.c_int]
    lib.app_stop.argtypes = [C.POINTER(AppResult)]
    return lib


def slot_ceiling(local, pk, n, slot_bytes, read_bytes, kernel_ms=None, reps=9):
    """tools/libceiling.so ceiling_slot_ms over the workload's own burst: the
    classify kernel's slot shape (8 lanes per slot, the frame's 16-B chunks,
    16 B stored per slot) with no parsing, and a plain read of the same
    n * slot_bytes; the dominant kernel's median dispatch beside them"""
    p = os.path.join(ROOT, "tools", "libceiling.so")
    if not os.path.exists(p):
        return None
    torch.cuda.synchronize()
    a, b = C.c_double(0.0), C.c_double(0.0)
    rc = C.CDLL(p).ceiling_slot_ms(C.c_int(local), C.c_void_p(pk.data_ptr()), C.c_ulonglong(n),
                                   C.c_uint(slot_bytes), C.c_uint(read_bytes), C.c_int(reps),
                                   C.byref(a), C.byref(b))
    if rc != 0:
        log(f"bench: ceiling_slot_ms failed (HIP error {rc})")
        return None
    out = dict(slot_ms=round(a.value, 4), stream_ms=round(b.value, 4),
               stream_gbs=round(n * slot_bytes / (b.value * 1e-3) / 1e9, 1))
    if kernel_ms:
        out.update(kernel_median_ms=kernel_ms, kernel_over_slot=round(kernel_ms / a.value, 3),
                   kernel_over_stream=round(kernel_ms / b.value, 3))
    return out


def hbm_read_ceiling(local, nbytes=4 << 30, reps=9):
    """this box's measured HBM read ceiling (GB/s) beside the 8 TB/s spec:
    tools/libceiling.so's plain coalesced read (tools/ceiling.hip), the
    fastest shape of tools/membw_large.hip; None if the tool is not built"""
    p = os.path.join(ROOT, "tools", "libceiling.so")
    if not os.path.exists(p):
        log("bench: tools/libceiling.so not built; hbm_read_ceiling_gbs = null")
        return None
    torch.cuda.empty_cache()
    g = C.c_double(0.0)
    rc = C.CDLL(p).ceiling_read_gbs(C.c_int(local), C.c_ulonglong(nbytes), C.c_int(reps),
                                    C.byref(g))
    if rc != 0:
        log(f"bench: ceiling_read_gbs failed (HIP error {rc})")
        return None
    return round(g.value, 1)


# ---------------------------------------------------------------------------
def e2e(name, local, batch, reps=20, inflight=4):
    """PCIe-inclusive rate of the host-buffer path: pinned host frames +
    descriptors -> H2D -> K1 -> verdicts D2H.  "sync": one burst at a time
    (rxg_classify_span).  "pipelined": rxg_submit with `inflight` bursts
    outstanding over the context's 3 staging slots, so copies in, the kernel
    and copies out of consecutive bursts overlap.  Reported in DESIGN.md,
    never as value."""
    w = rxdist.WORKLOADS[name]
    cfg = rxdist.gen_cfg(name)
    hp, ho, hl = R.gen_host(cfg, 0, batch, w["unit_log2"])
    # bytes the burst occupies (the packed layout ends before batch * slot_bytes)
    span = (int(ho[-1]) << w["unit_log2"]) + ((int(hl[-1]) + 63) & ~63) if cfg.packed \
        else batch * cfg.slot_bytes
    sets = []
    for _ in range(inflight):
        pk = torch.empty(span + 64, dtype=torch.uint8).pin_memory()
        off = torch.empty(batch, dtype=torch.int32).pin_memory()
        ln = torch.empty(batch, dtype=torch.int16).pin_memory()
        out = torch.empty(batch * 16, dtype=torch.uint8).pin_memory()
        pk.numpy()[:span] = hp[:span]
        off.numpy().view(np.uint32)[:] = ho
        ln.numpy().view(np.uint16)[:] = hl
        sets.append((pk, off, ln, out))
    ctx = R.Context(local, max_pkts=batch, max_bytes=span + 64)
    udp, tcb = R.gen_flows(cfg)
    ctx.flows_sync(udp, tcb)

    def args(k):
        pk, off, ln, out = sets[k % inflight]
        return (pk.data_ptr(), span, off.data_ptr(), ln.data_ptr(), batch, w["unit_log2"],
                out.data_ptr())
    for k in range(3):
        ctx.classify_span(*args(k))
    t0 = time.perf_counter()
    for k in range(reps):
        ctx.classify_span(*args(k))
    el_sync = (time.perf_counter() - t0) / reps
    tickets = []
    for k in range(inflight):  # warm the pipeline
        tickets.append(ctx.submit(*args(k)))
    ctx.wait(tickets[-1])
    tickets = [None] * inflight
    t0 = time.perf_counter()
    for k in range(reps):
        if tickets[k % inflight] is not None:
            ctx.wait(tickets[k % inflight])  # this buffer set's previous burst
        tickets[k % inflight] = ctx.submit(*args(k))
    for t in tickets:
        if t is not None:
            ctx.wait(t)
    el = (time.perf_counter() - t0) / reps
    frame_bytes = int(hl.astype(np.int64).sum())
    ok = sets[0][3].numpy().view(R.VERDICT_DTYPE)["rc"]
    ctx.close()
    h2d = span + 6 * batch
    return dict(workload=name, frames_per_burst=batch, bursts=reps, inflight=inflight,
                ms_per_burst=round(el * 1e3, 3), mpps=round(batch / el / 1e6, 1),
                h2d_gb_per_s=round(h2d / el / 1e9, 2),
                alg_gb_per_s=round((frame_bytes + 22 * batch) / el / 1e9, 2),
                sync_ms_per_burst=round(el_sync * 1e3, 3), sync_mpps=round(batch / el_sync / 1e6, 1),
                rc0_frac=round(float((ok == 0).mean()), 4))


def pcie_peaks(local, nbytes=256 << 20, reps=10):
    """pinned host <-> HBM copy rates on this box (the PCIe roofline of the
    host-buffer path): H2D alone, D2H alone, both at once on two streams"""
    dev = torch.device("cuda", local)
    h = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
    h2 = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
    d = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    d2 = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)

    def rate(fn):
        fn()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize(dev)
        return (time.perf_counter() - t0) / reps

    def both():
        with torch.cuda.stream(s1):
            d.copy_(h, non_blocking=True)
        with torch.cuda.stream(s2):
            h2.copy_(d2, non_blocking=True)
    t_h2d = rate(lambda: d.copy_(h, non_blocking=True))
    t_d2h = rate(lambda: h2.copy_(d2, non_blocking=True))
    t_both = rate(both)
    return dict(h2d_gb_per_s=round(nbytes / t_h2d / 1e9, 2), d2h_gb_per_s=round(nbytes / t_d2h / 1e9, 2),
                duplex_gb_per_s=round(2 * nbytes / t_both / 1e9, 2))


def sweep(ctx, names, steps, warmup, dev, only="", with_counts=False):
    """Tuning: every kernel variant, interleaved over rounds in one process
    (same data, same device), median and min of the per-round kernel time."""
    variants = [tuple(int(x) for x in v.split(",")) for v in only.split(";") if v] or \
        R.KERNEL_VARIANTS
    # a 5th field = resident blocks per CU cap
    variants = [v if len(v) == 5 else v + (0,) for v in variants]
    for nm in names:
        w = rxdist.WORKLOADS[nm]
        cfg = rxdist.gen_cfg(nm)
        n = w["n"]
        udp, tcb = R.gen_flows(cfg)
        ctx.flows_sync(udp, tcb)
        sh = torch.cuda.current_stream(dev).cuda_stream
        pk = torch.empty(n * cfg.slot_bytes + 64, dtype=torch.uint8, device=dev)
        off = torch.empty(n, dtype=torch.int32, device=dev)
        ln = torch.empty(n, dtype=torch.int16, device=dev)
        out = torch.empty(n * 16, dtype=torch.uint8, device=dev)
        cnt = torch.zeros(ctx.num_flows, dtype=torch.int64, device=dev) if with_counts else None
        R.gen_dev(cfg, 0, n, pk, off, ln, w["unit_log2"], stream=sh)
        torch.cuda.synchronize(dev)
        alg = int(ln.to(torch.int64).bitwise_and(0xFFFF).sum().item()) + 22 * n
        ok = []
        for v in variants:  # drop variants that are not compiled in
            ctx.tune(*v[:4])
            try:
                ctx.classify_dev(pk, off, ln, n, w["unit_log2"], w["len_hint"], out, cnt,
                                 stream=sh)
                ok.append(v)
            except R.RxgError as e:
                log(f"sweep {nm} variant={v}: skipped ({e})")
        variants = ok
        times = {v: [] for v in variants}
        for rnd in range(5):
            for v in variants:
                ctx.tune(*v[:4])
                ctx.tune_grid(v[4])
                for _ in range(warmup):
                    ctx.classify_dev(pk, off, ln, n, w["unit_log2"], w["len_hint"], out, cnt,
                                     stream=sh)
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for _ in range(steps):
                    ctx.classify_dev(pk, off, ln, n, w["unit_log2"], w["len_hint"], out, cnt,
                                     stream=sh)
                b.record()
                torch.cuda.synchronize(dev)
                times[v].append(a.elapsed_time(b) / steps)
        ctx.tune(0)
        ctx.tune_grid(0)
        for v in variants:
            t = sorted(times[v])
            med = t[len(t) // 2]
            log(f"sweep {nm}{' +counts' if with_counts else ''} variant={v}: median {med:.4f} ms min {t[0]:.4f} ms "
                f"-> {n / med / 1e3:.0f} Mpps, {alg / med / 1e6:.0f} GB/s")
        del pk, off, ln, out, cnt
        torch.cuda.empty_cache()


# ---------------------------------------------------------------------------
# The stdout line.  The driver parses a bounded tail of stdout (round 4's
# 21-KB line was cut mid-object and read as unparsed), so stdout carries a
# compact line of at most LINE_MAX bytes: the headline fields, roofline,
# cpu_baseline, the parity / digest booleans and one scalar summary per extra
# workload and socket mode.  The full result dict goes to the detail file.
LINE_MAX = 4096
DETAIL_PATH = os.path.join(ROOT, "gpurun_out", "bench_detail.json")


def write_detail(full):
    """the full result dict (per-burst arrays, phase maps, O0 / nproc legs,
    per_rank) as JSON in gpurun_out/ (BENCH_DETAIL overrides); returns the
    path, or None if it could not be written (reported on stderr)"""
    path = os.environ.get("BENCH_DETAIL", DETAIL_PATH)
    try:
        os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
        with open(path, "w") as f:
            json.dump(full, f, indent=1)
        log(f"bench: full detail in {path}")
        return path
    except OSError as e:
        log(f"bench: detail file not written ({e}); full line follows on stderr")
        log(json.dumps(full))
        return None


def _g(d, *ks):
    """d[k0][k1]... or None"""
    for k in ks:
        if not isinstance(d, dict) or k not in d:
            return None
        d = d[k]
    return d


def _wl_summary(r, peak=HBM_PEAK_GBS):
    """one extra workload as scalars"""
    s = dict(mpps=_g(r, "mpps"), gb_per_s=_g(r, "gbps"), ms_per_step=_g(r, "ms_per_step"),
             frac=round(r["gbps"] / peak, 4) if isinstance(r.get("gbps"), (int, float)) else None,
             kernel_median_ms=_g(r, "roofline", "kernel", "median_ms"),
             kernel_frac=_g(r, "roofline", "kernel", "frac"),
             traffic=_g(r, "roofline", "traffic"),
             parity_ok=(_g(r, "parity", "mismatches") == 0) if _g(r, "parity") else None,
             digest_ok=_g(r, "digest", "digest_ok"), counts_match=_g(r, "counts_match"),
             cpu_mpps=_g(r, "cpu_baseline", "value"),
             v8_frac=_g(r, "verdict8", "frac"), tx_frac=_g(r, "tx_cksum", "frac"),
             kernel_over_slot_shape=_g(r, "slot_shape_ceiling", "kernel_over_slot"),
             kernel_over_stream=_g(r, "slot_shape_ceiling", "kernel_over_stream"))
    return {k: (round(v, 4) if isinstance(v, float) else v) for k, v in s.items()
            if v is not None}


def _sock_summary(s):
    """one socket-API mode as scalars"""
    if "error" in s:
        return dict(error=str(s["error"])[:120])
    out = dict(mpps=_g(s, "mpps"), overlapped_mpps=_g(s, "overlapped", "mpps"),
               cpu_mpps=_g(s, "cpu_baseline", "mpps"),
               inplace_mpps=_g(s, "inplace", "mpps"),
               d2h_ms=_g(s, "rx_burst_phases_ms", "d2h"),
               app_lock_wait_ms=_g(s, "overlapped", "app_ms_per_burst", "lock_wait"),
               received_equal=_g(s, "overlapped", "received_equal"),
               pipelined_mpps=_g(s, "pipelined", "mpps"),
               inplace_pipelined_mpps=_g(s, "inplace_pipelined", "mpps"),
               overlapped_inplace_mpps=_g(s, "overlapped_inplace", "mpps"),
               overlapped_pipelined_inplace_mpps=_g(s, "overlapped_pipelined_inplace", "mpps"),
               overlapped_pipelined_mpps=_g(s, "overlapped_pipelined", "mpps"),
               pipelined_received_equal=_g(s, "overlapped_pipelined", "received_equal"))
    return {k: v for k, v in out.items() if v is not None}


def compact_line(full, limit=LINE_MAX):
    """the stdout line from the full result dict (see LINE_MAX)"""
    keep = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
            "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config", "gb_per_s",
            "ramp_ms")
    out = {k: full[k] for k in keep if k in full}
    rf = full.get("roofline") or {}
    out["roofline"] = {k: rf.get(k) for k in ("bound", "achieved", "peak", "unit", "frac",
                                               "traffic")}
    if rf.get("kernel"):
        out["roofline"]["kernel"] = {k: rf["kernel"].get(k) for k in ("name", "median_ms",
                                                                     "frac")}
    cb = full.get("cpu_baseline")
    if cb:
        out["cpu_baseline"] = dict(
            value=cb.get("value"), unit=cb.get("unit"), cores=cb.get("cores"),
            kind=cb.get("kind"),
            sample=(cb.get("sample_short") or cb.get("sample") or "")[:200],
            all_cores_mpps=_g(cb, "O2", "all_cores", "mpps"),
            all_cores_threads=_g(cb, "O2", "all_cores", "threads"),
            O0_mpps=_g(cb, "O0", "one_core", "mpps"), model=_g(cb, "host", "model"))
    else:
        out["cpu_baseline"] = None
    par = full.get("parity") or {}
    out["parity"] = dict(checked=par.get("checked"), mismatches=par.get("mismatches"))
    out["digest_ok"] = _g(full, "digest", "digest_ok")
    out["counts_match"] = full.get("counts_match")
    out["hbm_read_ceiling_gbs"] = full.get("hbm_read_ceiling_gbs")
    if "per_rank" in full:
        pr = full["per_rank"] or []
        ms = [p["ms_per_step"] for p in pr]
        out["ranks"] = dict(n=len(pr), rccl_nranks=full.get("rccl_nranks"),
                            ms_per_step_max=max(ms) if ms else None,
                            ms_per_step_min=min(ms) if ms else None,
                            frames_min=min((p["frames"] for p in pr), default=None),
                            frames_max=max((p["frames"] for p in pr), default=None),
                            allreduce_ms=full.get("allreduce_ms"),
                            allreduce_bytes=full.get("allreduce_bytes"))
    if full.get("verdict8"):
        v8 = full["verdict8"]
        out["verdict8"] = dict(mpps=v8.get("mpps"), frac=v8.get("frac"),
                               ok=bool(v8.get("equals_projection")) and v8.get("digest_ok")
                               is not False)
    if full.get("tx_cksum"):
        out["tx_cksum"] = {k: full["tx_cksum"].get(k) for k in ("mpps", "frac")}
    if full.get("e2e_pcie"):
        out["e2e_pcie_mpps"] = full["e2e_pcie"].get("mpps")
    c1 = full.get("cfg1")
    if c1:
        out["cfg1"] = dict(pcie_mpps=_g(c1, "pcie_inclusive", "mpps"),
                           device_mpps=_g(c1, "device_resident", "mpps"),
                           cpu_mpps=_g(c1, "cpu_baseline", "value"),
                           parity_ok=_g(c1, "parity", "mismatches") == 0)
    for k, v in full.items():
        if k.startswith("cfg") and k != "cfg1" and isinstance(v, dict):
            out[k] = _wl_summary(v)
    if full.get("socket_api"):
        out["socket_api"] = {m: _sock_summary(s) for m, s in full["socket_api"].items()}
    # over the limit (never expected): drop the optional parts, least
    # important first, and say so
    extra = [k for k in out if k.startswith("cfg") and k != "cfg1"]
    for drop in ["socket_api", "cfg1", "verdict8", "tx_cksum"] + extra[::-1]:
        if len(json.dumps(out, separators=(",", ":"))) < limit - 200:
            break
        if drop in out:
            out.pop(drop)
            out.setdefault("dropped", []).append(drop)
    return out


def build_line(names, results, steps, warmup, ramp_ms, world, ndev, collective, rccl_nranks=None,
               ceiling=None, cfg1=None, sock=None):
    """rank 0: the full result line (before compact_line) from the workloads'
    results; the first workload is the headline.  rccl_nranks: the rank count
    the RCCL communicator itself reports (rxg_group_size), None without one"""
    head = results[names[0]]
    line = {
        "metric": "Mpps (device-resident rx parse+cksum+classify, 64 B frames)",
        "value": round(head["mpps"], 2),
        "unit": "Mpps",
        "n_gpus": world,
        "steps": steps,
        "warmup": warmup,
        "ramp_ms": ramp_ms,
        "ms_per_step": round(head["ms_per_step"], 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (deterministic counter-based pktgen, generated in HBM; cfg1 "
                "through a pcap file)",
        "config": {"workload": f"{names[0]}: {head['desc']}",
                   "frames_per_step": head["frames_per_step"], "flows": head["nflows"],
                   "parallelism": f"rss-split x{world}" if world > 1 else "1 GPU",
                   "collective": collective,
                   # ranks time-slicing one GPU (a rehearsal of the N-rank logic on a
                   # one-GPU box): their step times measure the sharing, not the kernels
                   "ranks_share_gpus": bool(world > max(ndev, 1))},
        "gb_per_s": round(head["gbps"], 2),
        "roofline": head["roofline"],
        "cpu_baseline": head.get("cpu_baseline"),
        "parity": head["parity"],
        "digest": head["digest"],
        "kernel_ms_avg": round(head["kernel_ms_avg"], 4),
        "counts_ok": head["counts_ok"],
        "counts_match": head["counts_match"],
        "hbm_read_ceiling_gbs": ceiling,
        "librxgpu_sha256": lib_sha256()[:16],
    }
    if world > 1:
        line["rccl_nranks"] = rccl_nranks
        line["allreduce_ms"] = head["allreduce_ms"]
        line["allreduce_bytes"] = head["allreduce_bytes"]
        line["per_rank"] = head["per_rank"]
    if "verdict8" in head:
        line["verdict8"] = head["verdict8"]
    if "tx_cksum" in head:
        line["tx_cksum"] = head["tx_cksum"]
    if "e2e_pcie" in head:
        line["e2e_pcie"] = head["e2e_pcie"]
        line["pcie_peaks"] = head["pcie_peaks"]
    if cfg1:
        line["cfg1"] = cfg1
    if sock:
        line["socket_api"] = sock
    for nm in names[1:]:
        r = results[nm]
        line[nm] = {k: (round(v, 4) if isinstance(v, float) else v) for k, v in r.items()}
    return line


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # 50 steps: a 12-ms timed window at cfg2 (0.23 ms per burst), less exposed
    # to a single host-side hiccup than 20 (4.6 ms)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="cfg2,cfg3,cfg4,cfg5",
                    help="BASELINE configs to run; the first is the headline line (cfg2 = configs[1])")
    ap.add_argument("--no-cfg1", action="store_true",
                    help="skip BASELINE configs[0] (pcap, 1 flow; rank 0 at N = 1 only)")
    ap.add_argument("--cpu-budget", type=float, default=4.0,
                    help="seconds of oracle work per CPU-baseline leg (headline workload)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--parity-sample", type=int, default=4096,
                    help="verdicts per rank and workload checked against the oracle after the "
                         "timed steps (0 = none)")
    ap.add_argument("--variant", default="", help="force a kernel variant g,p,fpg (tuning)")
    ap.add_argument("--no-counts", action="store_true", help="skip per-flow counting (ablation)")
    ap.add_argument("--cu-split", type=int, default=0,
                    help="slab-count workloads: run the count stream on this many CUs of its own "
                         "and the classify on the rest (hipExtStreamCreateWithCUMask; 0 = off)")
    ap.add_argument("--count-stream-priority", type=int, default=0,
                    help="torch priority of the count stream (negative = higher; A/B)")
    ap.add_argument("--no-count-stream", action="store_true",
                    help="per-flow counts on the classify stream (rxg_classify_dev), not "
                         "overlapped with the next step (A/B)")
    ap.add_argument("--no-tx", action="store_true", help="skip timing the TX checksum kernel")
    ap.add_argument("--no-v8", action="store_true",
                    help="skip the steps with 8-B verdicts (rxg_classify_dev8)")
    ap.add_argument("--collective", default="rxg", choices=["rxg", "torch"],
                    help="N > 1 count all-reduce: rxg = RCCL through librxgpu's C ABI "
                         "(rxg_group); torch = torch.distributed's nccl (RCCL) backend")
    ap.add_argument("--backend", default="gloo", help="torch.distributed backend of the control "
                    "plane (rendezvous, barriers, max-over-ranks timing)")
    ap.add_argument("--e2e", action="store_true", help="also measure the PCIe-inclusive rate")
    ap.add_argument("--no-sockrate", action="store_true",
                    help="skip the socket-API rate (nstack_rx_burst + nrecvfrom/nrecv)")
    ap.add_argument("--sweep-variants", default="", help="';'-separated g,p,fpg,pipe list")
    ap.add_argument("--ramp-ms", type=float, default=200.0,
                    help="untimed clock ramp per workload before the warmup steps (ms of wall time)")
    ap.add_argument("--flow-load", type=int, default=0,
                    help="flow tables at load <= 2**-N (rxg_tune_flow_load; 0 = default)")
    ap.add_argument("--sweep-counts", action="store_true", help="sweep with per-flow counts on")
    ap.add_argument("--tune-tables", type=int, default=0,
                    help="rxg_tune_tables flags (A/B: 4 = RXG_TT_COUNT_2BUF, the round-4 two "
                         "count-index buffers)")
    ap.add_argument("--shard-gen", default="direct", choices=["direct", "split"],
                    help="N > 1: each rank generates its RSS shard directly (direct) or every "
                         "rank generates the global burst, splits it and gathers its shard "
                         "(split: the shards partition one burst; golden digest of its first n "
                         "frames)")
    ap.add_argument("--deadline", type=float, default=0.0,
                    help="N > 1 without a launcher: wall-clock limit of the whole run in seconds "
                         "(0 = 120 + 120 per workload); past it every rank is stopped")
    ap.add_argument("--sweep", default="", help="time every kernel variant on these workloads "
                    "(tuning; prints to stderr, no JSON line)")
    a = ap.parse_args()
    # stdout carries the one JSON line only: native libraries (gloo, RCCL, HIP)
    # print to fd 1 as well, so fd 1 is pointed at stderr and the line goes to
    # a private duplicate of the original stdout
    global JSON_OUT
    JSON_OUT = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    sys.stdout = sys.stderr

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = torch.cuda.device_count()
    log(f"bench: rank {rank} of {world} (local {local}, pid {os.getpid()}, {ndev} GPU(s) visible)")
    hang = os.environ.get("BENCH_TEST_HANG_RANK")  # test hook: this rank blocks forever
    if hang is not None and int(hang) == rank:
        stage(rank, "rendezvous (BENCH_TEST_HANG_RANK: blocked on purpose)")
        while True:
            time.sleep(60)
    if ndev == 0:
        # no GPU: the rank set and the rendezvous are still checked (gloo),
        # then every rank fails loudly; nothing is measured without the device
        if world > 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            stage(rank, "rendezvous")
            torch.distributed.init_process_group("gloo")
            t = torch.ones(1)
            torch.distributed.all_reduce(t)
            log(f"bench: rank {rank}: rendezvous ok, all_reduce saw {int(t.item())} ranks")
            torch.distributed.destroy_process_group()
        log(f"bench: rank {rank}: no GPU visible; librxgpu has no CPU path (exit 4)")
        sys.exit(4)
    if world > 1 and ndev < world:  # rehearsal with ranks sharing GPUs (never RCCL then)
        local = local % max(ndev, 1)
    group = nccl_group = None
    collective = None
    rccl_nranks = None
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        stage(rank, "rendezvous")
        torch.distributed.init_process_group(a.backend)
        if a.collective == "rxg" and ndev >= world:
            try:  # rank 0 makes the RCCL id, gloo hands it to every rank
                obj = [R.group_id() if rank == 0 else None]
                torch.distributed.broadcast_object_list(obj, src=0)
                stage(rank, "rxg_group_open (RCCL communicator)")
                group = R.Group(local, world, rank, obj[0])
                rccl_nranks = group.size()[0]
                log(f"rank {rank}: RCCL communicator reports {rccl_nranks} ranks")
                collective = "rccl (rxg_group_open / rxg_counts_allreduce, C ABI)"
            except Exception as e:  # reported in the line, never silent
                log(f"rank {rank}: rxg_group_open failed ({e}); using torch.distributed nccl")
                group = None
        if group is None:
            nccl_group = torch.distributed.new_group(
                backend="nccl" if ndev >= world else "gloo")
            collective = "torch.distributed " + ("nccl (rccl)" if ndev >= world else "gloo")
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    ctx = R.Context(local)
    if a.flow_load:
        ctx.tune_flow_load(a.flow_load)
    if a.tune_tables:
        ctx.tune_tables(a.tune_tables)
    global COUNTS, TX, RAMP_MS, COUNT_STREAM, V8, CS_PRIORITY, CU_SPLIT
    CS_PRIORITY = a.count_stream_priority
    CU_SPLIT = a.cu_split
    V8 = not a.no_v8
    RAMP_MS = a.ramp_ms
    COUNT_STREAM = not a.no_count_stream
    COUNTS = not a.no_counts
    TX = not a.no_tx
    if a.variant:
        ctx.tune(*[int(x) for x in a.variant.split(",")])
    if a.sweep:
        sweep(ctx, a.sweep.split(","), a.steps, a.warmup, dev, a.sweep_variants, a.sweep_counts)
        return
    cores = host_cores()
    oracle_threads = max(1, cores["threads"] // max(1, min(world, 8)))
    names = [s.strip() for s in a.workload.split(",") if s.strip()]
    results = {}
    for nm in names:
        stage(rank, f"{nm}: setup")
        coll = None
        if world > 1:
            u, t = R.gen_flows(rxdist.gen_cfg(nm))
            coll = collective_fn(group, nccl_group, len(u) + len(t))
        results[nm] = run_workload(nm, ctx, rank, world, a.steps, a.warmup, dev, coll,
                                   a.parity_sample, oracle_threads, a.shard_gen)
        log(nm, json.dumps({k: v for k, v in results[nm].items() if k != "desc"}))
    head = results[names[0]]

    if rank == 0 and world == 1 and not a.no_cpu:
        for i, nm in enumerate(names):
            results[nm]["cpu_baseline"] = cpu_baseline(nm, a.cpu_budget if i == 0
                                                       else a.cpu_budget / 2, cores)
    cfg1 = None
    if rank == 0 and world == 1 and not a.no_cfg1:
        cfg1 = run_cfg1(local, dev, a.steps, a.warmup, 0 if a.no_cpu else a.cpu_budget / 2, cores)
        log("cfg1", json.dumps(cfg1))
    sock = {}
    if rank == 0 and world == 1 and not a.no_sockrate:
        for nm in ("cfg2", "cfg3"):
            try:
                sock[nm] = socket_api(local, nm, 0 if a.no_cpu else a.cpu_budget / 2, cores,
                                      with_cpu=not a.no_cpu)
                log("socket_api", json.dumps(sock[nm]))
            except Exception as e:  # reported in the line, never silent
                sock[nm] = dict(error=repr(e))
                log(f"socket_api {nm} failed: {e!r}")
    ceiling = hbm_read_ceiling(local) if rank == 0 and world == 1 else None

    if a.e2e and rank == 0:
        pk = pcie_peaks(local)
        log("pcie", json.dumps(pk))
        results[names[0]]["pcie_peaks"] = pk
        for nm in names:
            r = e2e(nm, local, {"cfg2": 1 << 20, "cfg3": 1 << 16}.get(nm, 1 << 16))
            log("e2e", json.dumps(r))
            results[nm]["e2e_pcie"] = r

    parity_bad = sum(r["parity"]["mismatches"] for r in results.values()) + \
        sum(r["counts_match"] is False for r in results.values()) + \
        (cfg1["parity"]["mismatches"] if cfg1 else 0) + \
        sum(r["digest"]["digest_ok"] is False for r in results.values()) + \
        sum(("verdict8" in r and (not r["verdict8"]["equals_projection"]
                                  or r["verdict8"]["digest_ok"] is False)) for r in results.values())
    if rank == 0:
        line = build_line(names, results, a.steps, a.warmup, a.ramp_ms, world, ndev, collective,
                          rccl_nranks, ceiling, cfg1, sock)
        # stdout: the compact line (the driver parses a bounded tail of
        # stdout); every measured detail goes to the detail file
        path = write_detail(line)
        short = compact_line(line)
        short["detail"] = os.path.relpath(path, ROOT) if path else None
        print(json.dumps(short, separators=(",", ":")), file=JSON_OUT, flush=True)
    ctx.close()
    if group is not None:
        group.close()
    if world > 1:
        torch.distributed.destroy_process_group()
    if parity_bad:
        log(f"bench: {parity_bad} verdicts differ from the oracle")
        sys.exit(3)


if __name__ == "__main__":
    main()
