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
    # max over ranks: rank 1 "takes" 80.8 ms, so the job rate is 2 x its rate
    b = 65536
    assert abs(j["value"] - 2 * 20 * b / 80.8e-3 / 1e6) < 1e-3 * j["value"]
    # the start gate opened both windows together
    assert j["windows"]["start_gate"] == "shm" and j["windows_overlap"] >= 0.9
    assert 0 < j["value_union"] <= 2 * 20 * b / 80e-3 / 1e6 * 1.001
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


def test_eight_ranks_gate_overlap_and_config5_block():
    """The driver's 8-GPU command: 8 ranks, the shared-memory start gate
    opens every rank's window at once (each rank sleeps its fake time inside
    it, so the overlap is measured, not assumed): a run with overlap >= 0.9 and
    the union-window rate beside the max-own value; the configs[4] secondary
    (fw_lpm_1m: 1M + 1M, 256k batches, per-rule counters reduced over all
    ranks) rides the line with its reduction checked across 8 ranks."""
    r = run("--gpus", "8", "--dry-run", "--steps", "20", "--warmup", "5", "--repeats", "5", "--no-cpu",
            timeout=600)
    assert r.returncode == 0, r.stderr
    lines = json_lines(r.stdout)
    assert len(lines) == 1
    j = lines[0]
    assert j["n_gpus"] == 8 and len(j["config"]["ranks"]) == 8
    # overlap = (first end - last start) / the median own time: at most
    # 80 / 82.8 = 0.966 here (rank r sleeps 80 (1 + r/100) ms). Eight ranks
    # spin at the gate on this container's 8 CPUs beside pytest, so a rank
    # can lose a scheduler tick (a few ms) before it stamps its start: at
    # least one run within 5 ms of together, and the median within 17 ms
    # (on a GPU box the skew is microseconds: start_skew_us)
    assert max(j["windows"]["per_run"]["overlap"]) >= 0.9, j["windows"]
    assert j["windows_overlap"] >= 0.75, j["windows"]
    assert len(j["windows"]["per_run"]["overlap"]) == 5
    b = 65536
    # value: max over ranks (rank 7 takes 85.6 ms); union: never above every
    # rank running its packets in the fastest rank's time
    assert abs(j["value"] - 8 * 20 * b / 85.6e-3 / 1e6) < 1e-3 * j["value"]
    assert j["value_union"] <= 8 * 20 * b / 80e-3 / 1e6 * 1.001
    c5 = j["secondary"]["fw_lpm_1m"]
    assert c5["rule_counters"] and c5["rccl_init"] == ["ok"] * 8
    B = 262144
    assert c5["counter_reduce"]["ok"] and c5["counter_reduce"]["ranks"] == 8
    assert c5["counter_reduce"]["pkts_reduced_per_interval"] == [8 * 25 * B] + [8 * 20 * B] * 4
    assert c5["windows_overlap"] >= 0.75
    assert {"fw_lpm", "fw_lpm_imix", "fw_lpm_1m"} <= set(j["secondary"])


def test_start_gate_and_window_stats_in_process():
    """window_stats on hand-made windows: overlap, skew and the union rate."""
    import copdist
    w = [[(0, 1000)], [(100, 1100)]]          # two ranks, 100 ns apart, 1000 ns each
    st = copdist.window_stats(w, 2, 10)
    assert st["windows_overlap"] == 0.9 and st["start_skew_us_median"] == 0.1
    assert abs(st["value_union"] - 2 * 10 / 1100e-9 / 1e6) < 1e-3   # (rounded to 3 decimals)
    w = [[(0, 1000)], [(2000, 3000)]]         # windows that never met
    assert copdist.window_stats(w, 2, 10)["windows_overlap"] < 0
