"""bench.py --gpus N launches its own ranks (one process per GPU) when no
launcher set RANK/WORLD_SIZE: the rank spawn, the gloo rendezvous on
127.0.0.1, the barrier-bracketed max-over-ranks timing, the per-rank gather
and rank 0's single JSON line, with the GPU leg stubbed (--dry-run). Also
the one-GPU-per-rank guard: N ranks on fewer GPUs are refused unless
--allow-shared-gpu."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def run(*args, timeout=300):
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    return subprocess.run([sys.executable, BENCH, *args], capture_output=True, text=True, timeout=timeout, env=env)


def json_lines(out):
    return [json.loads(x) for x in out.splitlines() if x.startswith("{")]


def test_spawn_two_ranks_one_line():
    r = run("--gpus", "2", "--dry-run", "--steps", "20", "--warmup", "5", "--repeats", "3", "--cpu-budget", "0.3")
    assert r.returncode == 0, r.stderr
    lines = json_lines(r.stdout)
    assert len(lines) == 1, r.stdout          # rank 0 only
    j = lines[0]
    assert j["n_gpus"] == 2 and j["steps"] == 20
    ranks = j["config"]["ranks"]
    assert [x["rank"] for x in ranks] == [0, 1]
    assert sorted(x["device"] for x in ranks) == [0, 1]          # one device per rank
    # max over ranks: rank 1 "takes" 1.1 ms, so the job rate is 2 x its rate
    b = 65536
    assert abs(j["value"] - 2 * 20 * b / 1.1e-3 / 1e6) < 1e-3 * j["value"]
    assert ranks[0]["mpkt_s"] > ranks[1]["mpkt_s"]
    # the CPU baseline rides every N's line (N > 1 lines had none)
    cb = j["cpu_baseline"]
    assert cb["cores"] == 1 and cb["kind"] == "port" and cb["value"] > 0 and cb["unit"] == "Mpkt/s"


def test_refuses_ranks_sharing_a_gpu():
    r = run("--gpus", "2", "--dry-run", "--dry-run-devices", "1", "--steps", "4", "--warmup", "0", "--repeats", "1",
            "--no-cpu")
    assert r.returncode != 0
    assert "each rank needs its own GPU" in r.stderr
    assert not json_lines(r.stdout)


def test_allow_shared_gpu():
    r = run("--gpus", "2", "--dry-run", "--dry-run-devices", "1", "--allow-shared-gpu", "--steps", "4",
            "--warmup", "0", "--repeats", "1", "--no-cpu")
    assert r.returncode == 0, r.stderr
    j = json_lines(r.stdout)[0]
    assert [x["device"] for x in j["config"]["ranks"]] == [0, 0]


def test_world_size_must_match_gpus():
    env = dict(os.environ, RANK="0", LOCAL_RANK="0", WORLD_SIZE="1")
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--dry-run"], capture_output=True, text=True,
                       timeout=120, env=env)
    assert r.returncode != 0 and "WORLD_SIZE=1 but --gpus 2" in r.stderr


def test_two_ranks_rule_counter_workload_protocol():
    """The config-5 branches the 8-GPU run takes: the RCCL unique-id
    broadcast from rank 0, the per-interval counter reduction (gloo standing
    in for the RCCL all-reduce) checked and reported — not asserted — and
    each rank's RCCL init status in config.ranks."""
    r = run("--gpus", "2", "--dry-run", "--workload", "fw_lpm_1m", "--steps", "20", "--warmup", "5", "--repeats", "3",
            "--no-cpu")
    assert r.returncode == 0, r.stderr
    lines = json_lines(r.stdout)
    assert len(lines) == 1
    line = lines[0]
    assert [x["rccl_init"] for x in line["config"]["ranks"]] == ["ok", "ok"]
    red = line["counter_reduce"]
    B = 262144
    assert red["ok"] and red["pkts_reduced_per_interval"] == [2 * 25 * B, 2 * 20 * B, 2 * 20 * B]


def test_failing_rank_ends_the_others_fast():
    """One rank exits at start (as a table or device error would): the parent
    ends the rank left waiting in the gloo rendezvous and returns the failure
    at once, not after gloo's long timeout."""
    import time as _t
    t0 = _t.time()
    r = run("--gpus", "2", "--dry-run", "--dry-run-fail-rank", "1", "--steps", "4", "--warmup", "0", "--repeats", "1",
            timeout=120)
    assert r.returncode != 0
    assert _t.time() - t0 < 60
    assert "failed first" in r.stderr
