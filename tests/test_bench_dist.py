"""CPU tests of bench.py's N > 1 path (gloo, world_size 2).

Packet groups are independent codewords (ugo/fec.go:145-146), so ranks own
contiguous group ranges and nothing but the timing barrier and two scalar
reductions crosses ranks.  These tests drive bench.py's own launcher
(`bench.py --gpus N` starts the ranks as a child torch.distributed.run and
forwards rank 0's line) and its own coordination code (dist_setup,
rank_groups, clock_warmup, timed_region, reduce_max, all_ranks_ok) through
tests/_bench_rank_cpu.py, a torchrun target that stands the CPU oracle in for
each rank's GPU (checker only).
"""
import json
import os
import sys

import pytest

import bench
from ugo_amd.shard import partition

HERE = os.path.dirname(os.path.abspath(__file__))
RANK_SCRIPT = os.path.join(HERE, "_bench_rank_cpu.py")


def test_launcher_command_shape():
    cmd = bench.launcher_cmd(["--gpus", "4", "--steps", "20"], 4, 29512)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--nnodes=1" in cmd
    assert "--master-addr=127.0.0.1" in cmd and "--master-port=29512" in cmd
    i = cmd.index(os.path.abspath(bench.__file__))
    assert cmd[i + 1:] == ["--gpus", "4", "--steps", "20"], "the child gets the same arguments"


def test_main_dispatch(monkeypatch):
    calls = []
    monkeypatch.setattr(bench, "launch", lambda argv, n, **k: calls.append(("launch", n, list(argv))) or 0)
    monkeypatch.setattr(bench, "run_rank", lambda args: calls.append(("rank", args.gpus)))
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    bench.main(["--steps", "3"])  # --gpus 1: unchanged, runs in this process
    assert calls[-1] == ("rank", 1)
    with pytest.raises(SystemExit) as ex:
        bench.main(["--gpus", "2", "--steps", "3"])  # no torchrun environment: launches
    assert ex.value.code == 0 and calls[-1] == ("launch", 2, ["--gpus", "2", "--steps", "3"])
    monkeypatch.setenv("WORLD_SIZE", "2")  # inside torchrun: this process is a rank
    bench.main(["--gpus", "2"])
    assert calls[-1] == ("rank", 2)


def test_result_line_filter():
    assert bench.is_result_line('{"metric": "x", "value": 1}\n')
    assert not bench.is_result_line('{"other": 1}')
    assert not bench.is_result_line("rank 1 noise on stdout")
    assert not bench.is_result_line("{not json")
    # another rank's unterminated output sharing the pipe line
    assert bench.result_json('rank 1 noise{x}{"metric": "x", "value": 1}\n') == '{"metric": "x", "value": 1}'
    assert bench.result_json('{"metric": "x", "value": 1}rank 1 noise\n') == '{"metric": "x", "value": 1}'


@pytest.mark.parametrize("total", [1000, 7])
def test_two_ranks_through_bench_launcher(total, capfd, monkeypatch):
    """bench.launch starts 2 gloo ranks; rank 0's line is the only stdout line."""
    monkeypatch.setenv("BENCH_TEST_TOTAL", str(total))
    rc = bench.launch(["--gpus", "2"], 2, script=RANK_SCRIPT, timeout=240)
    out, err = capfd.readouterr()
    assert rc == 0, err[-2000:]
    lines = [ln for ln in out.splitlines() if ln.strip()]
    assert len(lines) == 1, out
    r = json.loads(lines[0])
    assert r["n_gpus"] == 2 and r["scaling"] == "strong" and r["total_groups"] == total
    assert r["tmax"] == 1.5, "max-over-ranks time reduction"
    assert r["max_rank"] == 1.0
    sizes = [partition(total, 2, k)[1] - partition(total, 2, k)[0] for k in range(2)]
    assert r["gmax"] == max(sizes)
    assert r["covered"] == total, "the last rank's range ends at the total"
    assert r["all_ok"] is True, "every rank's slice equals the single-process result"
    assert r["one_bad"] is False, "one failing rank makes all_ranks_ok false"
    assert r["elapsed_pos"] and r["cw_steps"] >= 15
    assert "rank 1 noise on stdout" in err, "other ranks' stdout goes to stderr"


def test_rank_groups_weak_and_strong():
    assert bench.rank_groups(0, 65536, 3, 8) == (3 * 65536, 65536, "weak", 8 * 65536)
    g0, G, sc, tot = bench.rank_groups(4194304, 65536, 7, 8)
    assert (g0, G, sc, tot) == (7 * 524288, 524288, "strong", 4194304)
    spans = [bench.rank_groups(10, 0, r, 3)[:2] for r in range(3)]
    assert spans == [(0, 3), (3, 3), (6, 4)]


def test_clock_warmup_waits_for_settled_steps():
    import itertools
    import time

    # step times fall for 6 chunks (the clock ramp), then settle
    durs = itertools.chain([0.004, 0.003, 0.0025, 0.002, 0.0015, 0.0012], itertools.repeat(0.001))
    cur = {"d": 0.0}

    def step():
        pass

    def sync():
        time.sleep(cur["d"])
        cur["d"] = next(durs)

    ms, steps, settled = bench.clock_warmup(step, sync, 1.0, chunk=1, max_ms=1000.0)
    assert settled and steps >= 8, (ms, steps)
    ms, steps, settled = bench.clock_warmup(step, lambda: time.sleep(0.002), 30.0, chunk=1)
    assert ms >= 30.0 and settled


def test_partition_covers_exactly_once():
    for total in (0, 1, 7, 65536, 4194304):
        for world in (1, 2, 3, 8):
            ranges = [partition(total, world, r) for r in range(world)]
            assert ranges[0][0] == 0 and ranges[-1][1] == total
            for (a0, a1), (b0, b1) in zip(ranges, ranges[1:]):
                assert a1 == b0 and a0 <= a1
            sizes = [b - a for a, b in ranges]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        partition(10, 2, 2)


def test_host_info_fields():
    info = bench.host_info()
    assert set(info) == {"cpu_model", "nproc", "affinity_cpus", "cgroup_cpu_quota", "cgroup_quota_file",
                         "usable_cpus", "go_toolchain"}
    assert info["go_toolchain"] in ("present", "absent") and info["affinity_cpus"] >= 1
    # the CPU baseline runs on every usable CPU: the affinity set, capped by a cgroup quota if one is set
    assert 1 <= info["usable_cpus"] <= info["affinity_cpus"]
    if info["cgroup_cpu_quota"] is not None:
        assert info["usable_cpus"] == max(1, min(info["affinity_cpus"], int(info["cgroup_cpu_quota"])))


def test_cgroup_quota_parsing(tmp_path, monkeypatch):
    """cpu.max (v2) along the process's cgroup path: the smallest quota wins."""
    root = tmp_path / "cg"
    (root / "a" / "b").mkdir(parents=True)
    (root / "cpu.max").write_text("max 100000\n")
    (root / "a" / "cpu.max").write_text("1600000 100000\n")
    (root / "a" / "b" / "cpu.max").write_text("3200000 100000\n")
    real_open = open

    def fake_open(path, *a, **k):
        path = str(path)
        if path == "/proc/self/cgroup":
            import io
            return io.StringIO("0::/a/b\n")
        if path.startswith("/sys/fs/cgroup"):
            path = str(root) + path[len("/sys/fs/cgroup"):]
        return real_open(path, *a, **k)

    monkeypatch.setattr("builtins.open", fake_open)
    q, src = bench.cgroup_cpu_quota()
    assert q == 16.0 and src.endswith("a/cpu.max")


def _fake_sysfs(root, cpus):
    """Two GPUs on two NUMA nodes, each node with half of `cpus`."""
    half = len(cpus) // 2 or 1
    nodes = {0: cpus[half:] or cpus, 1: cpus[:half]}
    for bdf, node in (("0000:0b:00.0", 1), ("0000:8c:00.0", 0)):
        d = os.path.join(root, "bus", "pci", "devices", bdf)
        os.makedirs(d)
        with open(os.path.join(d, "numa_node"), "w") as f:
            f.write(f"{node}\n")
    for node, cs in nodes.items():
        d = os.path.join(root, "devices", "system", "node", f"node{node}")
        os.makedirs(d)
        with open(os.path.join(d, "cpulist"), "w") as f:
            f.write(",".join(str(c) for c in cs) + "\n")
    return nodes


def test_numa_lookup_and_binding_on_a_fake_sysfs(tmp_path):
    from ugo_amd import numa

    cpus = sorted(os.sched_getaffinity(0))
    nodes = _fake_sysfs(str(tmp_path), cpus)
    assert numa.parse_cpulist("0-3,8,10-11\n") == [0, 1, 2, 3, 8, 10, 11]
    info = numa.gpu_numa_node(0, sysfs=str(tmp_path), bdf="0000:0b:00.0")
    assert info["numa_node"] == 1 and info["node_cpus"] == nodes[1]
    assert numa.gpu_numa_node(0, sysfs=str(tmp_path), bdf="0000:ff:00.0")["numa_node"] is None
    saved = os.sched_getaffinity(0)
    # a thread that exists before the binding (as HIP's, torch's and gloo's do) is bound too
    import threading

    go, tid = threading.Event(), []
    t = threading.Thread(target=lambda: (tid.append(threading.get_native_id()), go.wait(30)))
    t.start()
    while not tid:
        pass
    try:
        r = numa.bind_to_node(info)
        assert r["bound"] and sorted(os.sched_getaffinity(0)) == nodes[1]
        assert r["threads"] >= 2
        assert sorted(os.sched_getaffinity(tid[0])) == nodes[1]
    finally:
        go.set()
        t.join()
        numa.set_affinity_all_threads(saved)
    assert sorted(os.sched_getaffinity(0)) == sorted(saved)
    assert not numa.bind_to_node({"node_cpus": []})["bound"]


def test_host_path_coordination_two_ranks(tmp_path, capfd, monkeypatch):
    """bench.host_path_leg's multi-rank pieces on 2 gloo ranks: each rank finds
    its GPU's NUMA node in (a fake) sysfs and binds to that node's CPUs; a rep
    starts at a barrier and counts as the slowest rank's time; bytes are summed
    over ranks; every rank's placement reaches rank 0's line."""
    cpus = sorted(os.sched_getaffinity(0))
    nodes = _fake_sysfs(str(tmp_path), cpus)
    monkeypatch.setenv("BENCH_TEST_SYSFS", str(tmp_path))
    monkeypatch.setenv("BENCH_TEST_TOTAL", "100")
    rc = bench.launch(["--gpus", "2"], 2, script=RANK_SCRIPT, timeout=240)
    out, err = capfd.readouterr()
    assert rc == 0, err[-2000:]
    r = json.loads([ln for ln in out.splitlines() if ln.strip()][0])
    h = r["host"]
    assert 0.029 <= h["t_job"] < 0.5, "the job's time is the slower rank's (30 ms)"
    assert 0.0099 <= h["t_mine"] < h["t_job"], "rank 0's own time is its own (10 ms)"
    assert h["bytes"] == 3000
    pl = h["placement"]
    assert [x["rank"] for x in pl] == [0, 1]
    assert pl[0]["numa_node"] == 1 and pl[0]["cpus"] == nodes[1] and pl[0]["bound"]
    assert pl[1]["numa_node"] == 0 and pl[1]["cpus"] == nodes[0] and pl[1]["bound"]


def test_rx_tx_over_ranks_reports_the_slowest_rank(capfd, monkeypatch):
    """the rx_tx leg runs on every rank; rank 0's line keeps
    its own leg and adds, for every kernel time, the max over ranks and each
    rank's value (2 gloo ranks through bench.py's launcher)."""
    monkeypatch.setenv("BENCH_TEST_TOTAL", "100")
    rc = bench.launch(["--gpus", "2"], 2, script=RANK_SCRIPT, timeout=240)
    out, err = capfd.readouterr()
    assert rc == 0, err[-2000:]
    r = json.loads([ln for ln in out.splitlines() if ln.strip()][0])["rx_tx"]
    assert r["ranks"] == 2
    assert r["rx_in_order"]["rx_assemble_ms"] == 0.4  # rank 0's own
    assert r["max_over_ranks"]["rx_in_order.rx_assemble_ms"] == 1.4
    assert abs(r["max_over_ranks"]["tx.tx_assemble_ms"] - 0.3) < 1e-9
    assert [x["rx_in_order.rx_assemble_ms"] for x in r["per_rank"]] == [0.4, 1.4]
