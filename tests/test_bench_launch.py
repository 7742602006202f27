"""bench.py --gpus N starts N rank processes by itself (CPU, no GPU here).

The driver runs `python3 bench.py --gpus N ...` for its 1/2/4/8-GPU curve.
Without a launcher, bench.py must start N ranks (RANK / LOCAL_RANK /
WORLD_SIZE / MASTER_* set, one per GPU: the multi-queue split the reference's
README assumes, README.md:13, of its single rx queue, netfamily.c:38-39) and
relay their status; under a launcher, --gpus must equal WORLD_SIZE.  On this
GPU-less box every rank checks the rendezvous over gloo and then fails loudly
(exit 4): there is no CPU path to measure."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env_extra=None, timeout=240):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra or {})
    env["HIP_VISIBLE_DEVICES"] = env.get("HIP_VISIBLE_DEVICES", "")
    return subprocess.run([sys.executable, BENCH] + args, env=env, capture_output=True,
                          text=True, timeout=timeout)


def _no_gpu():
    import torch
    return torch.cuda.device_count() == 0


def test_gpus_2_spawns_two_ranks_without_a_launcher():
    if not _no_gpu():
        import pytest
        pytest.skip("GPU present: the spawn is exercised by the real bench")
    r = _run(["--gpus", "2", "--backend", "gloo", "--steps", "1", "--warmup", "0"])
    err = r.stderr
    assert "bench: launched 2 ranks" in err, err
    for k in range(2):
        assert f"bench: rank {k} of 2" in err, err
        assert f"bench: rank {k}: rendezvous ok, all_reduce saw 2 ranks" in err, err
    assert "bench: rank exit codes [4, 4]" in err, err
    assert r.returncode == 4, (r.returncode, err)
    assert r.stdout.strip() == ""  # no JSON line without a measurement


def test_gpus_must_match_launcher_world_size():
    r = _run(["--gpus", "4", "--steps", "1"], env_extra=dict(WORLD_SIZE="2", RANK="0",
                                                              LOCAL_RANK="0"))
    assert r.returncode == 2, r.stderr
    assert "--gpus 4 but the launcher started WORLD_SIZE=2" in r.stderr


def test_gpus_1_is_one_process():
    if not _no_gpu():
        import pytest
        pytest.skip("GPU present")
    r = _run(["--gpus", "1", "--steps", "1"])
    assert "launched" not in r.stderr
    assert "bench: rank 0 of 1" in r.stderr
    assert r.returncode == 4, r.stderr


def test_hung_rank_ends_the_run_at_the_deadline_naming_its_stage():
    """a rank that never reaches the rendezvous (here rank 1,
    blocked on purpose by the BENCH_TEST_HANG_RANK hook) leaves rank 0 waiting
    in it; past --deadline the launcher prints each rank's last stage,
    stops both and exits 124 instead of hanging the driver's run"""
    if not _no_gpu():
        import pytest
        pytest.skip("GPU present")
    r = _run(["--gpus", "2", "--backend", "gloo", "--steps", "1", "--deadline", "15"],
             env_extra=dict(BENCH_TEST_HANG_RANK="1"), timeout=120)
    err = r.stderr
    assert r.returncode == 124, (r.returncode, err)
    assert "deadline 15 s passed; rank 1" in err, err
    assert "last stage: rendezvous (BENCH_TEST_HANG_RANK: blocked on purpose)" in err, err
    assert "deadline 15 s passed; rank 0" in err and "last stage: rendezvous" in err, err
    assert r.stdout.strip() == ""
