#!/usr/bin/env python3
"""bench.py -- device-resident FEC encode + reconstruct throughput on MI355X.

Metric (BASELINE.json): "FEC encode+decode GiB/s device-resident, (10+3)x1350B
groups; %HBM roofline".  One step = one pass of the hot path over one batch:
  1. ugo_fec_encode       -- Encoder.Encode (ugo/fec.go:238) on every group
  2. ugo_fec_reconstruct  -- Encoder.Reconstruct (ugo/fec.go:202) on every group
                             with exactly 2 distinct erased shards (uniform over
                             the 78 patterns, BASELINE configs[2])
Inputs are resident in HBM before the timed region (synthetic, device-generated
random bytes).  Steps alternate between 2 independent batches (--batches), so
every step works on a batch none of whose lines sit in the Infinity Cache --
the state a fresh batch of packets arrives in.  Algorithmic bytes per group
(BASELINE.md): encode (d+p)*S, reconstruct (d+e)*S; value = sum over ranks /
max-over-ranks time, in GiB/s.

Warm-up has two parts: a clock warm-up that runs untimed steps until at least
--clock-warmup-ms of load has passed and the last chunks of steps agree within
2 % (the clocks take ~20 ms of load to settle, so a step count alone is not a
warm-up), then the --warmup steps the driver asks for.  The timed region is
exactly --steps steps.

Multi-GPU: `python bench.py --gpus N` (N > 1, no torchrun environment) starts
N rank processes itself -- a child `torch.distributed.run` on 127.0.0.1, before
anything in this process touches a GPU -- and forwards rank 0's JSON line.
Packet groups are independent codewords (ugo/fec.go:145-146), so each rank
owns its own batch (weak scaling, default) or a contiguous 1/N slice of
--total-groups (strong scaling; BASELINE configs[3] is --total-groups 4194304),
and no collective touches the data path.  The only cross-rank traffic is the
timing barrier, one max-reduction and one all-ok reduction, which run over
gloo on the host (--dist-backend): they are control, not data, so RCCL has
nothing to carry.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--groups G]
                       [--total-groups T]
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "FEC encode+decode GiB/s device-resident, (10+3)×1350B groups; %HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak, GB/s (MI355X_MICROARCH.md)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one per GPU); > 1 without a torchrun environment launches them")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=50,
                    help="untimed steps after the clock warm-up")
    ap.add_argument("--clock-warmup-ms", type=float, default=200.0,
                    help="untimed load before the --warmup steps: at least this long, and until the last 3 "
                         "chunks of steps agree within 2%% (capped at 10x this)")
    ap.add_argument("--groups", type=int, default=65536, help="groups per GPU (weak scaling)")
    ap.add_argument("--total-groups", type=int, default=0, help="if set: strong scaling over this many groups")
    ap.add_argument("--data-shards", type=int, default=10)
    ap.add_argument("--parity-shards", type=int, default=3)
    ap.add_argument("--shard-size", type=int, default=1350)
    ap.add_argument("--pitch", type=int, default=0, help="row pitch in HBM (default: shard size rounded to 16)")
    ap.add_argument("--out-pitch", type=int, default=0,
                    help="row pitch of the reconstruct_into output batch (default: the batch pitch)")
    ap.add_argument("--out-layout", choices=["planar", "grouped"], default="planar",
                    help="reconstruct_into output batch: planar [p][G][pitch] or grouped [G][p][pitch]")
    ap.add_argument("--erasures", type=int, default=2)
    ap.add_argument("--batches", type=int, default=2,
                    help="rotate the steps over this many independent batches per GPU (step k works on batch "
                         "k mod B). With B >= 2 every step meets a cold batch, as a fresh batch of packets is: "
                         "none of its lines are in the 256-MB Infinity Cache. B = 1 re-runs one batch, and the "
                         "cache then absorbs part of the rewritten parity (DESIGN.md §4)")
    ap.add_argument("--row-pad", type=int, default=0,
                    help="planar layout: bytes added between consecutive row streams (row stride G*pitch + this)")
    ap.add_argument("--layout", choices=["planar", "interleaved"], default="planar",
                    help="planar = shard-major [d+p][G][pitch] batch; interleaved = [G][d+p][pitch]")
    ap.add_argument("--decode", choices=["inplace", "into"], default="into",
                    help="inplace = ugo_fec_reconstruct_strided (erased rows rebuilt inside the batch); into = "
                         "ugo_fec_reconstruct_into (erased rows written to a separate [p][G][pitch] output batch, "
                         "the fresh buffers klauspost's Reconstruct gives ugo's nil shards)")
    ap.add_argument("--seed", type=int, default=0x5EED)
    ap.add_argument("--dist-backend", choices=["gloo", "nccl"], default="gloo",
                    help="process group for the timing barrier and reductions (no data-path collective)")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=8.0,
                    help="per leg of the CPU baseline (all cores, 1 core); the 2-erasure leg gets half")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU baseline threads; 0 = every usable CPU: min(affinity set, cgroup cpu.max quota)")
    ap.add_argument("--cpu-simd", type=int, default=-1,
                    help="CPU baseline SIMD level: -1 best available, 0 scalar, 1 AVX2, 2 AVX-512 GFNI")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--c4-total-groups", type=int, default=4194304,
                    help="strong leg after the main line: BASELINE configs[3] -- this many groups split over the "
                         "ranks (contiguous ranges), one cold batch per rank; 0 = off")
    ap.add_argument("--c4-steps", type=int, default=10, help="timed steps of the strong leg")
    ap.add_argument("--no-host-path", action="store_true",
                    help="skip the PCIe-inclusive host_path leg (every rank, NUMA-bound): pinned-host encode / "
                         "reconstruct of (10+3)x1350 x 65,536 and (32+8)x9000 x 8,192 groups, the host-memory RX "
                         "and TX paths, the PCIe ceilings (and, at N = 1, the per-call leg)")
    ap.add_argument("--no-rx-tx", action="store_true",
                    help="skip the rx_tx leg (every rank): RX / TX assembly, data-only recovery and packet decode "
                         "kernels with their ceilings")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"),
                    help="per-launch HBM bytes from rocprofv3 PMC passes (tools/pmc_traffic.py)")
    return ap.parse_args(argv)


# ------------------------------------------------------------------ launcher
def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launcher_cmd(argv, nproc: int, port: int, script: str = None):
    """The child command `bench.py --gpus N` runs: one process per rank, the
    rendezvous on 127.0.0.1 (the container hostname may not resolve)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
            "--master-addr=127.0.0.1", f"--master-port={port}", script or os.path.abspath(__file__)] + list(argv)


def result_json(line: str):
    """The result object in one line of the ranks' shared stdout, or None.
    Ranks write to one pipe, so another rank's output can share the line,
    before or after the object: it is parsed from the first '{' it starts at."""
    dec = json.JSONDecoder()
    k = line.find("{")
    while k >= 0:
        try:
            obj, end = dec.raw_decode(line, k)
            if isinstance(obj, dict) and "metric" in obj:
                return line[k:end]
        except ValueError:
            pass
        k = line.find("{", k + 1)
    return None


def is_result_line(line: str) -> bool:
    return result_json(line) is not None


def launch(argv, nproc: int, script: str = None, timeout: float = None) -> int:
    """Runs the ranks as a child process (never exec: this process may not
    replace itself) and forwards rank 0's JSON line as this process's only
    stdout line; everything else the child prints goes to stderr.  Returns the
    child's exit code."""
    cmd = launcher_cmd(argv, nproc, free_port(), script)
    print("bench.py: launching " + " ".join(cmd), file=sys.stderr, flush=True)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, env=env, text=True)
    n_lines = 0
    try:
        for line in proc.stdout:
            res = result_json(line)
            if res is not None and n_lines == 0:
                sys.stdout.write(res + "\n")
                sys.stdout.flush()
                n_lines += 1
                rest = line.replace(res, "", 1)
                if rest.strip():
                    sys.stderr.write(rest if rest.endswith("\n") else rest + "\n")
            else:
                sys.stderr.write(line)
        rc = proc.wait(timeout=timeout)
    except BaseException:
        proc.kill()
        proc.wait()
        raise
    if rc == 0 and n_lines != 1:
        print("bench.py: the ranks exited without a result line", file=sys.stderr)
        return 1
    return rc


# ---------------------------------------------------- rank-side coordination
def dist_setup(backend: str):
    """(rank, local_rank, world) from the torchrun environment; joins the
    process group when world > 1."""
    from ugo_amd.shard import dist_env

    rank, local_rank, world = dist_env()
    if world > 1:
        import torch.distributed as dist

        # one node, rendezvous on the loopback address: keep gloo's sockets on
        # the loopback device too (the container hostname may not resolve)
        if backend == "gloo" and os.environ.get("MASTER_ADDR", "127.0.0.1") in ("127.0.0.1", "localhost"):
            os.environ.setdefault("GLOO_SOCKET_IFNAME", "lo")
        import datetime

        # a rank that fails surfaces as an error within minutes instead of
        # leaving the others in a collective for gloo's default 30
        dist.init_process_group(backend, init_method="env://", timeout=datetime.timedelta(seconds=600))
    return rank, local_rank, world


def rank_groups(total_groups: int, groups: int, rank: int, world: int):
    """(first group, groups on this rank, scaling, total groups).  Strong
    scaling: a contiguous 1/world slice of total_groups; weak: `groups` each."""
    from ugo_amd.shard import partition

    if total_groups:
        g0, g1 = partition(total_groups, world, rank)
        return g0, g1 - g0, "strong", total_groups
    return rank * groups, groups, "weak", groups * world


def barrier(world: int):
    if world > 1:
        import torch.distributed as dist

        dist.barrier()


def reduce_max(values, world: int):
    """Element-wise max over ranks of a list of floats (host tensors, so any
    backend carries it)."""
    import torch

    t = torch.tensor([float(v) for v in values], dtype=torch.float64)
    if world > 1:
        import torch.distributed as dist

        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return t.tolist()


def reduce_sum(values, world: int):
    """Element-wise sum over ranks of a list of numbers (host tensors)."""
    import torch

    t = torch.tensor([float(v) for v in values], dtype=torch.float64)
    if world > 1:
        import torch.distributed as dist

        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t.tolist()


def all_ranks_ok(ok: bool, world: int) -> bool:
    import torch

    t = torch.tensor([int(bool(ok))], dtype=torch.int64)
    if world > 1:
        import torch.distributed as dist

        dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(t.item())


def timed_region(step, steps: int, sync, world: int) -> float:
    """Exactly `steps` steps bracketed by barrier + device synchronize on both
    sides; returns this rank's wall time from the start barrier to its own
    last step done (reduce_max gives the job's: the slowest rank's).  The
    closing barrier is outside the clock: its latency (a gloo round over all
    ranks) is not step time, and at --steps 20 (a ~7 ms region) it would be
    a visible share of it."""
    barrier(world)
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    elapsed = time.perf_counter() - t0
    barrier(world)
    return elapsed


def clock_warmup(step, sync, min_ms: float, chunk: int = 5, tol: float = 0.02, max_ms: float = None):
    """Untimed steps until at least min_ms of load has run and the last 3
    chunks of `chunk` steps agree within `tol` (or max_ms has passed).
    Returns (elapsed ms, steps run, settled)."""
    max_ms = 10 * min_ms if max_ms is None else max_ms
    times = []
    n = 0
    sync()
    t_start = time.perf_counter()
    while True:
        t0 = time.perf_counter()
        for _ in range(chunk):
            step()
        sync()
        t1 = time.perf_counter()
        n += chunk
        times.append(t1 - t0)
        el = (t1 - t_start) * 1e3
        last = times[-3:]
        settled = len(last) == 3 and max(last) <= (1 + tol) * min(last)
        if (el >= min_ms and settled) or el >= max_ms:
            return el, n, settled


# ------------------------------------------------------------- CPU baseline
def cgroup_cpu_quota():
    """CPUs the cgroup CPU controller grants this process: the smallest
    cpu.max quota/period (cgroup v2) or cfs_quota_us/cfs_period_us (v1) along
    the process's cgroup path up to the root, as a float; None if no quota is
    set (or the files are not readable).  Returns (cpus, source)."""
    best, src = None, None

    def consider(q, per, path):
        nonlocal best, src
        if q > 0 and per > 0 and (best is None or q / per < best):
            best, src = q / per, path

    try:
        with open("/proc/self/cgroup") as f:
            lines = f.read().splitlines()
    except OSError:
        lines = []
    for line in lines:
        parts = line.split(":", 2)
        if len(parts) != 3:
            continue
        _, ctrls, rel = parts
        if ctrls == "":  # v2 unified hierarchy
            roots = ["/sys/fs/cgroup"]
            fname = "cpu.max"
        elif "cpu" in ctrls.split(","):
            roots = ["/sys/fs/cgroup/cpu,cpuacct", "/sys/fs/cgroup/cpu"]
            fname = None
        else:
            continue
        for root in roots:
            rel_parts = [p for p in rel.split("/") if p]
            for k in range(len(rel_parts), -1, -1):
                d = os.path.join(root, *rel_parts[:k])
                try:
                    if fname:
                        with open(os.path.join(d, fname)) as f:
                            q, per = f.read().split()[:2]
                        if q != "max":
                            consider(float(q), float(per), os.path.join(d, fname))
                    else:
                        with open(os.path.join(d, "cpu.cfs_quota_us")) as f:
                            q = float(f.read().strip())
                        with open(os.path.join(d, "cpu.cfs_period_us")) as f:
                            per = float(f.read().strip())
                        consider(q, per, os.path.join(d, "cpu.cfs_quota_us"))
                except (OSError, ValueError):
                    continue
    return best, src


def host_info():
    """CPU model, machine CPU count, this process's CPU share (affinity set and
    cgroup quota) and whether a Go toolchain exists (the reference is Go;
    BASELINE.md's CPU plan)."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        share = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        share = os.cpu_count() or 1
    go = shutil.which("go")
    quota, quota_src = cgroup_cpu_quota()
    usable = share if quota is None else max(1, min(share, int(quota)))
    return {"cpu_model": model, "nproc": os.cpu_count(), "affinity_cpus": share,
            "cgroup_cpu_quota": None if quota is None else round(quota, 2), "cgroup_quota_file": quota_src,
            "usable_cpus": usable, "go_toolchain": "present" if go else "absent"}


def cpu_baseline(args, d, p, S, n):
    """The CPU oracle timed on this host's cores (rank 0, N = 1, after the GPU
    work).  Main figure: BASELINE configs[0] -- 1,024 groups of (10+3)x1350,
    Encode of every group, then 1 uniformly random erased shard per group and
    Reconstruct, each group one call as ugo/fec.go:196-217 (input) and
    :228-243 (calcECC) make them -- on all cores of this process's share and
    on 1 core.  Secondary: the bench's own 2-erasure workload on 4,096 groups.
    oracle/rs_oracle.c restates the upstream algorithm with the upstream
    library's SIMD strategy (AVX-512 GFNI affine or AVX2 nibble tables, per-
    pattern inverse cache).  The Go reference needs a Go toolchain, which
    the box lacks (host_info probes for one)."""
    import numpy as np

    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import rs_ref  # checker / CPU baseline only

    rs_ref.load_c_oracle()
    info = host_info()
    level = rs_ref.set_simd(args.cpu_simd)
    threads = info["usable_cpus"] if args.cpu_threads <= 0 else max(1, min(args.cpu_threads, info["usable_cpus"]))
    rng = np.random.default_rng(args.seed)

    base = rng.integers(0, 256, size=(1024, n, S), dtype=np.uint8)

    def sample(erasures):
        """One instance's own batch: a copy of one random base batch (instances
        never share memory) and its own uniformly random erasure pattern."""
        G = base.shape[0]
        erased = rng.random((G, n)).argsort(axis=1)[:, :erasures]
        masks = np.full(G, (1 << n) - 1, np.uint64)
        for j in range(erasures):
            masks &= ~(np.uint64(1) << erased[:, j].astype(np.uint64))
        return base.copy(), masks

    def leg(samples, erasures, seconds):
        """One worker thread per (batch, masks) sample, each a single-threaded
        oracle loop over its own batch (ctypes releases the GIL): the aggregate
        rate of len(samples) concurrent FEC instances, as a server runs one
        per connection.  Per-call thread fan-out over 1,024 groups would time
        thread start-up instead of coding."""
        import threading

        passes = [0] * len(samples)
        stop = threading.Event()

        def work(k):
            sh, masks = samples[k]
            while not stop.is_set():
                rs_ref.c_encode(d, p, sh, threads=1)
                rc, _ = rs_ref.c_reconstruct(d, p, sh, masks, threads=1)
                assert rc == 0
                passes[k] += 1

        ths = [threading.Thread(target=work, args=(k,)) for k in range(len(samples))]
        t0 = time.perf_counter()
        for t in ths:
            t.start()
        time.sleep(seconds)
        stop.set()
        for t in ths:
            t.join()
        el = time.perf_counter() - t0
        G = samples[0][0].shape[0]
        per_pass = G * ((d + p) * S + (d + erasures) * S)
        return round(per_pass * sum(passes) / el / 2**30, 4), sum(passes), el

    try:
        c0 = [sample(1) for _ in range(threads)]
        # per call on 1 core (the drop-in per-group path's CPU figure),
        # timed FIRST, before the all-core leg can leave the cgroup's quota
        # throttled: the C loop makes one Encode / Reconstruct per group, no
        # ctypes in between; 1 s of untimed calls first (clocks up)
        sh, masks = c0[0]
        t_end = time.perf_counter() + 1.0
        while time.perf_counter() < t_end:
            rs_ref.c_encode(d, p, sh, threads=1)
            rs_ref.c_reconstruct(d, p, sh, masks, threads=1)
        per = {"encode": [], "reconstruct_1loss": []}
        for _ in range(40):
            t0 = time.perf_counter()
            rs_ref.c_encode(d, p, sh, threads=1)
            t1 = time.perf_counter()
            rs_ref.c_reconstruct(d, p, sh, masks, threads=1)
            t2 = time.perf_counter()
            per["encode"].append((t1 - t0) / sh.shape[0] * 1e6)
            per["reconstruct_1loss"].append((t2 - t1) / sh.shape[0] * 1e6)
        per_us = {k: round(sorted(v)[len(v) // 2], 3) for k, v in per.items()}
        v_one, n_one, t_one = leg(c0[:1], 1, args.cpu_baseline_seconds)
        v_all, n_all, t_all = leg(c0, 1, args.cpu_baseline_seconds)
        # the pair time the steady single-core rate implies (agrees with per_us within ~10%)
        pair_bytes = (d + p) * S + (d + 1) * S
        pair_us_steady = round(pair_bytes / (v_one * 2**30) * 1e6, 3)
        del c0
        c2 = [sample(args.erasures) for _ in range(threads)]
        v_two, n_two, t_two = leg(c2, args.erasures, args.cpu_baseline_seconds / 2)
    finally:
        rs_ref.set_simd(0)
    simd = rs_ref.SIMD_NAMES[level]
    out = {"value": v_all, "unit": "GiB/s", "cores": threads, "kind": "port",
           "sample": f"BASELINE configs[0]: 1024 groups ({d}+{p})x{S}B, Encode every group then 1 uniformly "
                     f"random erased shard per group and Reconstruct, one group per call (ugo/fec.go:196-217, "
                     f":228-243); {threads} concurrent instances (one thread each, own batch): {n_all} passes in "
                     f"{t_all:.1f}s; oracle/rs_oracle.c "
                     f"[{simd}], a C restatement of the klauspost algorithm and its SIMD strategy (the Go "
                     f"reference cannot run: go toolchain {info['go_toolchain']})",
           "single_core": {"value": v_one, "unit": "GiB/s", "cores": 1, "passes": n_one,
                           "seconds": round(t_one, 2), "per_group_us": per_us,
                           "pair_us_per_group": round(per_us["encode"] + per_us["reconstruct_1loss"], 3),
                           "pair_us_from_steady_rate": pair_us_steady,
                           "note": "per_group_us timed before the all-core leg (no throttled quota); "
                                   "pair_us_from_steady_rate = (encode + 1-loss reconstruct bytes per group) / "
                                   "this leg's GiB/s"},
           "two_erasure": {"value": v_two, "unit": "GiB/s", "cores": threads, "passes": n_two,
                           "seconds": round(t_two, 2),
                           "sample": f"{threads} instances x 1024 groups, encode + {args.erasures}-erasure "
                                     f"reconstruct (the bench's own workload)"},
           "simd": simd}
    out.update(info)
    return out


# -------------------------------------------------------------- GPU ranks
def make_masks(G, n, e, seed, device):
    """Presence masks with exactly e distinct erased shards per group."""
    import torch

    gen = torch.Generator(device="cpu").manual_seed(seed)
    keys = torch.rand((G, n), generator=gen)
    erased = keys.argsort(dim=1)[:, :e]  # e distinct indices, uniform over C(n, e)
    masks = torch.full((G,), (1 << n) - 1, dtype=torch.int64)
    for j in range(e):
        masks ^= (1 << erased[:, j]).to(torch.int64)
    return masks.to(device), erased


def kernel_pass(enc, step, steps, sync):
    """Kernel-timing pass (`roofline`, `kernels`): `steps` steps with the
    library's launch timing on -- each launch issued with hipExtLaunchKernel
    start/stop events (ugo_fec_timing_begin), which carry the dispatch's own
    timestamps on the launch stream.  The events cost ~5 us per kernel
    boundary (tools/gap_probe.py: 374.8 vs 364.6 us per step), so no `value`
    is taken from this pass.  Returns (encode ms, reconstruct ms per step,
    this pass's wall seconds)."""
    import numpy as np

    enc.timing_begin(4 * steps + 16)
    sync()
    t1 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    wall = time.perf_counter() - t1
    recs, _untimed = enc.timing_end()
    kid = recs["kernel"]
    n_enc = int((kid == 1).sum())
    n_dec = int(np.isin(kid, (2, 3)).sum())
    assert n_enc >= steps and n_dec >= steps, (n_enc, n_dec)
    enc_ms = float(recs["ms"][kid == 1].sum()) / steps
    dec_ms = float(recs["ms"][np.isin(kid, (2, 3))].sum()) / steps  # apply (+ k_prepare for d+p > 16)
    return enc_ms, dec_ms, wall


def kernel_stats(enc_ms, dec_ms, enc_bytes, dec_bytes, payload):
    def one(ms, b):
        return {"avg_ms": round(ms, 5), "bytes_per_launch": b, "GBps": round(b / (ms * 1e-3) / 1e9, 1),
                "payload_GBps": round(payload / (ms * 1e-3) / 1e9, 1),
                "frac": round(b / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}

    return {"encode": one(enc_ms, enc_bytes), "reconstruct": one(dec_ms, dec_bytes)}


def strong_leg(args, enc, rank, world, dev, stream):
    """BASELINE configs[3]: --c4-total-groups (4,194,304) groups of the bench's
    code split over the ranks in contiguous ranges (strong scaling: the total
    is fixed as N grows), one batch per rank in the planar layout -- at these
    sizes (9-74 GB per GPU) every step is cold without rotating batches.  Same
    step as the main line (encode + reconstruct_into), a timed region with
    barrier + synchronize and max over ranks, a kernel-timing pass, and a
    full-size round trip (every output equals the erased row it rebuilds; the
    erased rows stay in the batch, reconstruct_into never reads them --
    tests/test_large_batches.py zeroes them first at this size)."""
    import torch

    from ugo_amd.shard import partition

    d, p, S = args.data_shards, args.parity_shards, args.shard_size
    n, e = d + p, args.erasures
    pitch = args.pitch or (S + 15) // 16 * 16
    total = args.c4_total_groups
    g0, g1 = partition(total, world, rank)
    G = g1 - g0
    gen = torch.Generator(device=dev).manual_seed(args.seed + 0xC4 + g0)
    sh = torch.randint(0, 256, (n, G, pitch), dtype=torch.uint8, device=dev, generator=gen)
    masks, erased = make_masks(G, n, e, args.seed + 0xC4 + 1000 + rank, dev)
    out = torch.zeros((p, G, pitch), dtype=torch.uint8, device=dev)

    def step():
        enc.encode_batch(sh, shard_size=S, stream=stream, shard_major=True)
        enc.reconstruct_into(sh, masks, out, shard_size=S, stream=stream, shard_major=True)

    sync = torch.cuda.synchronize
    for _ in range(2):
        step()
    sync()
    elapsed = timed_region(step, args.c4_steps, sync, world)
    enc_ms, dec_ms, _ = kernel_pass(enc, step, args.c4_steps, sync)
    elapsed, enc_ms, dec_ms = reduce_max([elapsed, enc_ms, dec_ms], world)
    view = sh.transpose(0, 1)
    gi = torch.arange(G, device=dev)
    es = erased.sort(dim=1).values.to(dev)
    ok = all(bool(torch.equal(out[j, :, :S], view[gi, es[:, j], :S])) for j in range(e))
    ok = all_ranks_ok(ok, world)
    # the ceiling at this size: the encode's compute-free twin on this same
    # batch (after the round trip: it writes wrong parity on purpose)
    twin = None
    if d == 10 and p == 3:
        try:
            import ctypes

            import numpy as np

            ms = np.zeros(4, np.float32)
            bases = (ctypes.c_void_p * 1)(sh.data_ptr())
            if probe_library().ugo_probe_encode_twin(bases, 1, G, S, pitch, sh.stride(0), 4, stream.cuda_stream,
                                                     ms.ctypes.data) == 0:
                twin = float(ms[1:].mean())
        except Exception:  # noqa: BLE001
            twin = None
        twin = reduce_max([twin if twin is not None else -1.0], world)[0]
    step_bytes = total * (n * S + (d + e) * S)
    res = {"workload": f"BASELINE configs[3]: {total} groups ({d}+{p})x{S}B total, strong over {world} rank(s): "
                       f"{G} groups on rank 0, one cold planar batch per rank, encode + {e}-erasure "
                       f"reconstruct_into",
           "total_groups": total, "groups_per_rank": G, "steps": args.c4_steps, "scaling": "strong",
           "value": round(step_bytes * args.c4_steps / elapsed / 2**30, 3), "unit": "GiB/s",
           "ms_per_step": round(elapsed / args.c4_steps * 1e3, 4),
           "kernels_rank_max": kernel_stats(enc_ms, dec_ms, G * n * S, G * (d + e) * S, G * d * S),
           "verify_round_trip_full_size": ok}
    if twin and twin > 0:
        res["encode_twin_ms"] = round(twin, 4)
        res["encode_frac_of_twin"] = round(twin / enc_ms, 4)
        res["note"] = ("below the 65,536-group rate at N = 1: the loss is the access pattern's own at this "
                       "footprint (HBM placement of a 74-GB batch), not the kernel -- encode_twin_ms is the "
                       "encode's compute-free twin on this same batch, and the encode runs at encode_frac_of_twin "
                       "of it (builder runs: profiles/r2/tlbprobe_r2.jsonl, profiles/r2/c4/c4_same_box_*.json, "
                       "profiles/r3/capprobe_4m*.jsonl)")
    del sh, out, masks, view
    torch.cuda.empty_cache()
    return res


def host_path_leg(args, dev_index, rank=0, world=1, reps=3):
    """The PCIe-inclusive rate north_star asks for (the path starts and ends in
    host memory: UDP socket buffers, /root/reference/ugo/conn.go:387-406), on
    every rank at once.  Each rank first binds itself to the
    NUMA node of its GPU (ugo_amd/numa.py: hipDeviceGetPCIBusId -> sysfs
    numa_node -> that node's CPUs), then allocates its pinned batches
    (ugo_fec_host_alloc), group-major as a packet ring lays them out:
      * (10+3)x1350 x 65,536 groups: ugo_fec_encode_host, then 2 uniformly
        random erasures per group and ugo_fec_reconstruct_host;
      * (32+8)x9000 x 8,192 groups (BASELINE configs[4]): encode, then a
        uniformly random 0..8 erasures per group (mixed patterns) and
        reconstruct.
    The encode stages through device buffers (H2D of the data rows -> kernel
    -> D2H of the parity rows, pipelined over 3 streams); the reconstruct of a
    pinned batch runs zero-copy on its device mapping.  Each
    call: 1 untimed, then `reps` timed, each rep started by a barrier over the
    ranks; the rep's time is the max over ranks, the reported time the median
    rep.  Aggregate GB/s = all ranks' bytes / that time.  Verified on every
    rank: each rebuilt batch equals the encoded batch it was erased from
    (compared on the device).  The process's CPU affinity is restored after."""
    import numpy as np
    import torch

    from ugo_amd import fec, numa

    dev = torch.device("cuda", dev_index)
    place = numa.gpu_numa_node(dev_index)
    saved = os.sched_getaffinity(0)
    bound = numa.bind_to_node(place)
    res = {"ranks": world}
    all_ok = True
    try:
        for d, p, S, G, mixed in ((10, 3, 1350, 65536, False), (32, 8, 9000, 8192, True)):
            # every rank makes the same collective calls whatever fails locally
            # (a failure is recorded and the rank's calls become no-ops), so a
            # failing rank cannot leave the others waiting in a barrier
            n = d + p
            pitch = (S + 15) // 16 * 16
            st = {"err": None}
            enc = raw = buf = ref = None
            masks = ne = None
            rcs = []

            def guarded(fn):
                def g():
                    if st["err"] is None:
                        try:
                            fn()
                        except Exception as ex:  # noqa: BLE001
                            st["err"] = repr(ex)[:200]
                return g

            def setup():
                nonlocal enc, raw, buf
                enc = fec.New(d, p, device=dev_index)
                raw = fec.host_alloc(G * n * pitch)
                buf = raw.reshape(G, n, pitch)
                gen = torch.Generator(device=dev).manual_seed(args.seed + d + 7919 * rank)
                torch.from_numpy(buf).copy_(torch.randint(0, 256, (G, n, pitch), dtype=torch.uint8, device=dev,
                                                          generator=gen))

            def erase():
                nonlocal ref, masks, ne
                ref = torch.from_numpy(buf).to(dev)
                rng = np.random.default_rng(args.seed + 7 * d + 104729 * rank)
                ranks_ = rng.random((G, n)).argsort(axis=1).argsort(axis=1)  # rank of row r in a random order
                ne = rng.integers(0, p + 1, G) if mixed else np.full(G, args.erasures)
                erased = ranks_ < ne[:, None]  # ne[g] distinct rows, uniform
                masks = np.zeros(G, np.uint64)
                for r in range(n):
                    masks |= (~erased[:, r]).astype(np.uint64) << np.uint64(r)
                gi, ri = np.nonzero(erased)
                buf[gi, ri] = 0

            try:
                guarded(setup)()
                enc_call = guarded(lambda: enc.encode_host(buf, S))
                enc_call()  # untimed
                t_enc, t_enc_mine = timed_reps(enc_call, reps, world)
                guarded(erase)()
                rec_call = guarded(lambda: rcs.append(enc.reconstruct_host(buf, masks, S)))
                rec_call()  # untimed
                t_rec, t_rec_mine = timed_reps(rec_call, reps, world)
                ok = st["err"] is None and all(rc == 0 for rc in rcs) and bool(
                    torch.equal(torch.from_numpy(buf).to(dev)[:, :, :S], ref[:, :, :S]))
                all_ok = all_ok and ok
                ref = None
                b_enc = G * n * S
                b_rec = 0 if ne is None else int((ne > 0).sum()) * d * S + int(ne.sum()) * S
                b_rec_all = int(reduce_sum([b_rec], world)[0])  # erasure counts differ by rank
                key = f"{d}+{p}x{S}"
                res[key] = {
                    "groups_per_rank": G, "erasures": "U[0,%d] per group" % p if mixed else f"{args.erasures} per group",
                    "encode_ms": round(t_enc * 1e3, 3), "encode_GBps": round(world * b_enc / t_enc / 1e9, 2),
                    "encode_pcie_GBps": round(world * G * (d * pitch + p * S) / t_enc / 1e9, 2),
                    "reconstruct_ms": round(t_rec * 1e3, 3),
                    "reconstruct_GBps": round(b_rec_all / t_rec / 1e9, 2),
                    "reconstruct_pcie_GBps": round(b_rec_all / t_rec / 1e9, 2),
                    "rank0_alone_encode_ms": round(t_enc_mine * 1e3, 3),
                    "rank0_alone_reconstruct_ms": round(t_rec_mine * 1e3, 3),
                    "verify_round_trip": ok}
                if st["err"]:
                    res[key]["error_rank0"] = st["err"]
            finally:
                if raw is not None:
                    fec.host_free(raw)
                if enc is not None:
                    enc.close()
        # the RX and TX paths from host memory to host memory, same binding
        rxtx, ok_rxtx = host_rxtx_cases(args, dev_index, rank, world, max(reps, 5))
        res.update(rxtx)
        all_ok = all_ok and ok_rxtx
    finally:
        numa.set_affinity_all_threads(saved)
    res["verify_all_ranks"] = all_ranks_ok(all_ok, world)
    me = {"rank": rank, "device": dev_index, "pci_bus_id": place["pci_bus_id"], "numa_node": place["numa_node"],
          "bound": bound.get("bound", False), "cpus": bound.get("cpus")}
    res["placement"] = gather_objects(me, world)
    res["note"] = ("pinned host batches, group-major, allocated after each rank bound itself to its GPU's NUMA node; "
                   "times: median over reps of the max over ranks (each rep starts at a barrier); GBps = all ranks' "
                   "algorithmic bytes ((d+p)*S encode, (d+e)*S per lossy group reconstruct) / that time; pcie_GBps "
                   "= bytes crossing PCIe (encode: d padded rows in + p rows out, staged; reconstruct: d survivor "
                   "rows in + e rows out, zero-copy); bound: sum of per-GPU PCIe links and host DRAM (DESIGN.md §6)")
    return res


def pcie_ceiling(dev, world, nbytes=1 << 30, reps=5):
    """The per-GPU PCIe ceiling measured in this run, every rank at once (each
    rep starts at a barrier, max over ranks): a 1-GiB pinned host buffer
    (ugo_fec_host_alloc) copied to the device, back, and both directions at once
    on two streams, with the copy calls the host paths use (hipMemcpyAsync,
    libugoprobe's ugo_probe_pcie).  GB/s are per GPU; "bidirectional" counts
    both directions' bytes.  (Round 5's first lines timed torch tensor copies,
    whose two directions never overlapped -- over this memory or with torch's
    own pinned tensors: 57.1-57.6 GB/s "both at once".)"""
    import ctypes

    import numpy as np
    import torch

    from ugo_amd import fec

    raw = [fec.host_alloc(nbytes), fec.host_alloc(nbytes)]
    try:
        dbuf = [torch.empty(nbytes, dtype=torch.uint8, device=dev) for _ in range(2)]
        lib = probe_library()
        ms = np.zeros(3, np.float32)
        barrier(world)
        rc = lib.ugo_probe_pcie(raw[0].ctypes.data, raw[1].ctypes.data, dbuf[0].data_ptr(), dbuf[1].data_ptr(),
                                nbytes, reps, ms.ctypes.data)  # medians over reps
        if rc != 0:
            raise RuntimeError(f"ugo_probe_pcie: {rc}")
        tmax = reduce_max([float(x) for x in ms], world)
        out = {"h2d_GBps": round(nbytes / (tmax[0] * 1e-3) / 1e9, 2),
               "d2h_GBps": round(nbytes / (tmax[1] * 1e-3) / 1e9, 2),
               "bidirectional_GBps": round(2 * nbytes / (tmax[2] * 1e-3) / 1e9, 2),
               "note": f"{nbytes >> 20} MiB pinned <-> device per copy (hipMemcpyAsync, one stream per direction; "
                       "two-way: the best over the ordered pairs of four streams), every rank at once, max over "
                       "ranks, per GPU"}
        del dbuf
        return out
    finally:
        for x in raw:
            fec.host_free(x)


def host_rxtx_cases(args, dev_index, rank, world, reps):
    """The host-memory RX and TX paths (include/ugo_fec.h
    ugo_fec_rx_recover_host / ugo_fec_tx_assemble_host), on every rank at once,
    pinned buffers allocated after the NUMA binding:
      * RX (ugo/listener.go:48 -> ugo/conn.go:387-406 -> ugo/fec.go:107-226): a
        recvmmsg-shaped ring of 65,536 (10+3) groups minus 5 % uniform loss,
        in seqid order, 1476-B RC4 packets in 1488-B slots plus uint16 lengths,
        in; the lost data shards of every lossy group out (compact);
      * TX (ugo/conn.go:643-685, :634): 65,536 groups of 10 full 1476-B data
        packets in 1488-B slots in; 13 RC4 wire packets per group out.
    Each call: 1 untimed, `reps` timed (barrier, max over ranks, median).
    Verified against the device-resident path on the same inputs.  wire_GBps =
    all ranks' wire bytes (RX: packets received; TX: packets sent) / time;
    pcie_GBps = bytes crossing this GPU's link / time, beside the measured
    per-GPU ceiling."""
    import numpy as np
    import torch

    from ugo_amd import fec

    d, p, n, S, pitch, slot, G = 10, 3, 13, 1470, 1472, 1488, 65536
    dev = torch.device("cuda", dev_index)
    res, ok_all = {}, True
    st = {"err": None}

    def guarded(fn):
        def g():
            if st["err"] is None:
                try:
                    fn()
                except Exception as ex:  # noqa: BLE001
                    st["err"] = repr(ex)[:200]
        return g

    try:
        res["pcie_ceiling"] = pcie_ceiling(dev, world)
    except Exception as ex:  # noqa: BLE001
        res["pcie_ceiling"] = {"error": repr(ex)[:200]}
    pad_b = fec.rc4_keystream(b"1234567890123456", slot)
    pad = torch.frombuffer(bytearray(pad_b), dtype=torch.uint8).to(dev)
    enc = fec.New(d, p, device=dev_index)
    bufs = []
    try:
        # ---- RX
        box = {}

        def rx_setup():
            gen = torch.Generator(device=dev).manual_seed(args.seed + 0x5B + 7919 * rank)
            seq = torch.arange(G * n, device=dev, dtype=torch.int64)
            seq = seq[torch.rand(G * n, device=dev, generator=gen) >= 0.05]
            npk = seq.numel()
            w = torch.randint(0, 256, (npk, slot), dtype=torch.uint8, device=dev, generator=gen)
            hdr = torch.zeros((npk, 6), dtype=torch.uint8, device=dev)
            for b in range(4):
                hdr[:, b] = ((seq >> (8 * b)) & 0xFF).to(torch.uint8)
            hdr[:, 4] = torch.where(seq % n < d, 0xF1, 0xF2).to(torch.uint8)
            w[:, :6] = hdr ^ pad[:6]
            ring = fec.host_alloc(npk * slot).reshape(npk, slot)
            lens = fec.host_alloc(npk * 2).view(np.uint16)
            out = fec.host_alloc(G * p * pitch).reshape(G * p, pitch)
            bufs.extend([ring, lens.view(np.uint8), out])
            torch.from_numpy(ring).copy_(w)
            lens[:] = 1476
            box.update(ring=ring, lens=lens, out=out, npk=npk, dring=w)

        def rx_call():
            box["r"] = enc.rx_recover_host(box["ring"], box["lens"], S, G, pad=pad_b, out=box["out"], max_out=G)

        guarded(rx_setup)()
        guarded(rx_call)()
        rx_reps = []
        t_rx, t_rx_mine = timed_reps(guarded(rx_call), reps, world, rx_reps)
        ok = False
        if st["err"] is None:
            # reference: the device-resident path on the same ring
            bat = torch.empty((n, G, pitch), dtype=torch.uint8, device=dev)
            pr = torch.zeros(G, dtype=torch.int64, device=dev)
            enc.rx_assemble(box["dring"], torch.from_numpy(box["lens"].view(np.int16)).to(dev), bat, pr,
                            shard_size=S, pad=pad)
            lst, cnt = enc.lossy_groups(pr, data_only=True)
            lo = torch.empty((G, p, pitch), dtype=torch.uint8, device=dev)
            enc.reconstruct_list(bat, pr, lst, cnt, lo, shard_size=S, data_only=True)
            k = int(cnt.item())
            nrec, index, out, _ = box["r"]
            # ugo's `recovered` order: entries ascending, each entry's lost data rows ascending
            pm = pr[lst[:k].long()]
            ed, okg = lost_and_recoverable(pm, d, n)
            lost = (((pm[:, None] >> torch.arange(d, device=dev)) & 1) == 0) & okg[:, None]
            jj, rr = torch.nonzero(lost, as_tuple=True)
            want_index = lst[:k].long()[jj] * n + rr
            want_rows = lo[:k][(torch.arange(p, device=dev)[None, :] < ed[:, None]) & okg[:, None]]
            ok = nrec == int(jj.numel()) and bool(np.array_equal(index[:nrec].astype(np.int64),
                                                                  want_index.cpu().numpy()))
            ok = ok and bool(torch.equal(torch.from_numpy(out[:nrec, :S]).to(dev), want_rows[:, :S]))
            del bat, pr, lo
        ok_all = ok_all and ok
        # the zero-copy alternative: rx_assemble reads the pinned ring over PCIe itself (no DMA
        # staging), then the same lossy list + list reconstruct, and the D2H of the recovered rows
        zc = {}

        def rx_zero_copy():
            ring_t = torch.from_numpy(box["ring"])
            lens_t = torch.from_numpy(box["lens"].view(np.int16))
            if "zb" not in zc:
                zc.update(zb=torch.empty((n, G, pitch), dtype=torch.uint8, device=dev),
                          zp=torch.zeros(G, dtype=torch.int64, device=dev),
                          zl=torch.empty(G, dtype=torch.int32, device=dev),
                          zc=torch.empty(1, dtype=torch.int32, device=dev),
                          zo=torch.empty((G, p, pitch), dtype=torch.uint8, device=dev),
                          pad=pad)
            zc["zp"].zero_()
            enc.rx_assemble(ring_t, lens_t, zc["zb"], zc["zp"], shard_size=S, pad=zc["pad"])
            enc.lossy_groups(zc["zp"], data_only=True, out=zc["zl"], count=zc["zc"])
            enc.reconstruct_list(zc["zb"], zc["zp"], zc["zl"], zc["zc"], zc["zo"], shard_size=S, data_only=True)
            k = int(zc["zc"].item())  # entry form: k entries x p row slots cross PCIe
            torch.from_numpy(box["out"][:k * p]).copy_(zc["zo"][:k].reshape(k * p, pitch))
            torch.cuda.synchronize(dev)

        t_zc = None
        if st["err"] is None:
            guarded(rx_zero_copy)()
            t_zc, _ = timed_reps(guarded(rx_zero_copy), reps, world)
            zc.clear()
        npk = box.get("npk", 0)
        nrec = box["r"][0] if "r" in box else 0
        wire_bytes = int(reduce_sum([npk * 1476], world)[0])
        pcie = npk * (slot + 2) + nrec * S
        res["rx_host"] = {
            "groups_per_rank": G, "packets_per_rank": npk, "loss": 0.05, "rc4": True, "recovered_shards_rank0": nrec,
            "rx_ms": round(t_rx * 1e3, 3), "wire_GBps": round(wire_bytes / t_rx / 1e9, 2),
            "pcie_GBps_per_gpu": round(pcie / t_rx / 1e9, 2), "rank0_alone_ms": round(t_rx_mine * 1e3, 3),
            "pcie_bound_ms": _r3(pcie_bound_ms(res.get("pcie_ceiling"), npk * (slot + 2), nrec * S, False)),
            "of_pcie_bound": _r3(pcie_bound_ms(res.get("pcie_ceiling"), npk * (slot + 2), nrec * S, False),
                                 t_rx * 1e3),
            "rep_ms": [round(t * 1e3, 2) for t in rx_reps],
            "zero_copy_ring_ms": None if t_zc is None else round(t_zc * 1e3, 3),
            "zero_copy_note": "rx_assemble reading the pinned ring in place, then the public lossy list + "
                              "entry-form list reconstruct, D2H of every entry's p row slots",
            "zero_copy_wire_GBps": None if t_zc is None else round(wire_bytes / t_zc / 1e9, 2),
            "verify_vs_device_path": ok,
            "path": "pinned ring -> H2D in >= 4 chunks on one copy stream, each chunk assembled as it lands -> "
                    "lossy-group list with row offsets -> data-only list reconstruct, row-compact -> D2H of "
                    "the recovered shards only (ugo's `recovered` order)"}
        box.clear()
        # ---- TX
        tb = {}

        def tx_setup():
            gen = torch.Generator(device=dev).manual_seed(args.seed + 0x7C + 7919 * rank)
            dp = torch.randint(0, 256, (G * d, slot), dtype=torch.uint8, device=dev, generator=gen)
            pk = fec.host_alloc(G * d * slot).reshape(G * d, slot)
            ln = fec.host_alloc(G * d * 2).view(np.uint16)
            wire = fec.host_alloc(G * n * slot).reshape(G * n, slot)
            wl = fec.host_alloc(G * n * 2).view(np.uint16)
            bufs.extend([pk, ln.view(np.uint8), wire, wl.view(np.uint8)])
            torch.from_numpy(pk).copy_(dp)
            ln[:] = 1476
            tb.update(pk=pk, ln=ln, wire=wire, wl=wl, dp=dp)

        def tx_call():
            enc.tx_assemble_host(tb["pk"], tb["ln"], tb["wire"], tb["wl"], pad=pad_b, max_len=1476)

        guarded(tx_setup)()
        for _ in range(3):  # untimed: a context's first host TX calls run slow (50 / 30 / 30 ms, then 26)
            guarded(tx_call)()
        tx_reps = []
        t_tx, t_tx_mine = timed_reps(guarded(tx_call), reps, world, tx_reps)
        ok = False
        if st["err"] is None:
            dw = torch.empty((G * n, slot), dtype=torch.uint8, device=dev)
            dwl = torch.empty(G * n, dtype=torch.int16, device=dev)
            enc.tx_assemble(tb["dp"], torch.from_numpy(tb["ln"].view(np.int16)).to(dev), dw, dwl, pad=pad,
                            max_len=1476)
            ok = bool(torch.equal(torch.from_numpy(tb["wire"]).to(dev)[:, :1476], dw[:, :1476])) and bool(
                np.array_equal(tb["wl"], dwl.cpu().numpy().view(np.uint16)))
            del dw, dwl
        ok_all = ok_all and ok
        res["tx_host"] = {
            "groups_per_rank": G, "packets_out_per_rank": G * n, "rc4": True, "tx_ms": round(t_tx * 1e3, 3),
            "wire_GBps": round(world * G * n * 1476 / t_tx / 1e9, 2),
            "pcie_GBps_per_gpu": round(G * (d + n) * slot / t_tx / 1e9, 2), "rank0_alone_ms": round(t_tx_mine * 1e3, 3),
            "pcie_bound_ms": _r3(pcie_bound_ms(res.get("pcie_ceiling"), G * d * (slot + 2), G * n * (slot + 2))),
            "of_pcie_bound": _r3(pcie_bound_ms(res.get("pcie_ceiling"), G * d * (slot + 2), G * n * (slot + 2)),
                                 t_tx * 1e3),
            "rep_ms": [round(t * 1e3, 2) for t in tx_reps],
            "verify_vs_device_path": ok,
            "path": "pinned data packets -> H2D -> tx_assemble -> D2H of the wire packets, group chunks through "
                    "4 device stages, the H2D copies on one stream, each chunk's kernel and D2H on a second, "
                    "joined by events (default stream classes)"}
        tb.clear()
        if st["err"]:
            res["rxtx_error_rank0"] = st["err"]
    finally:
        for b in bufs:
            fec.host_free(b)
        enc.close()
        torch.cuda.empty_cache()
    return res, ok_all and st["err"] is None


def _r3(x, div=None):
    """round(x, 3), or x / div rounded; None passes through."""
    if x is None:
        return None
    return round(x / div if div else x, 3)


def pcie_bound_ms(ceiling, h2d_bytes, d2h_bytes, overlap=True):
    """The least time the measured link allows for h2d_bytes in and d2h_bytes
    out: with overlap, both directions streaming at once -- each at half the
    measured two-way rate while both run, then the longer one alone at its
    one-way rate; without (the output depends on all the input, as RX's
    recovered rows do), one after the other at the one-way rates.  None
    without a ceiling."""
    try:
        h2d, d2h, both = ceiling["h2d_GBps"] * 1e9, ceiling["d2h_GBps"] * 1e9, ceiling["bidirectional_GBps"] * 1e9
    except (KeyError, TypeError):
        return None
    if not overlap:
        return (h2d_bytes / h2d + d2h_bytes / d2h) * 1e3
    if not d2h_bytes:
        return h2d_bytes / h2d * 1e3
    if not h2d_bytes:
        return d2h_bytes / d2h * 1e3
    t1 = min(h2d_bytes, d2h_bytes) / (both / 2)  # both directions at once
    rest = max(h2d_bytes, d2h_bytes) - t1 * both / 2
    return (t1 + rest / (h2d if h2d_bytes > d2h_bytes else d2h)) * 1e3


def timed_reps(call, reps, world, all_out=None):
    """`reps` calls, each started by a barrier over the ranks and timed on each
    rank; returns (median over reps of the max over ranks, this rank's own
    median): the job's time for one call when all ranks run it at once.
    all_out (a list): receives the max-over-ranks time of every rep."""
    ts = []
    for _ in range(reps):
        barrier(world)
        t0 = time.perf_counter()
        call()
        ts.append(time.perf_counter() - t0)
    mine = sorted(ts)[len(ts) // 2]
    mx = reduce_max(ts, world)
    if all_out is not None:
        all_out.extend(mx)
    return sorted(mx)[len(ts) // 2], mine


def gather_objects(obj, world):
    """[obj of rank 0, ..., obj of rank world-1] (gloo/host)."""
    if world <= 1:
        return [obj]
    import torch.distributed as dist

    out = [None] * world
    dist.all_gather_object(out, obj)
    return out


def per_call_leg(args, dev_index):
    """The drop-in route's latency (north_star: unchanged Encode / Reconstruct
    signatures, ugo/fec.go:202,238): one (10+3) group per call, as the cgo shim
    of INTEGRATION.md §2 makes it -- a pinned stage at the 16-B pitch, groups =
    1 -- with the 1470-B calcECC window for Encode and ugo's 1476-B buffers and
    one lost data shard for Reconstruct.  Each call is made through the C-ABI
    (ctypes: ~1 us of Python call overhead included) 2,000 times after 200
    untimed, median per call; first on the launch path, then with the per-call
    service on (ugo_fec_service_start).  Verified: the service's parity and
    rebuilt shard equal the launch path's.  Then what a resident service costs
    everyone else (interference): the bench step and a PCIe-inclusive encode,
    each timed alternately with and without a resident service block."""
    import ctypes

    import numpy as np

    from ugo_amd import fec

    d, p = 10, 3
    n = d + p
    lib = fec.load_library()
    enc = fec.New(d, p, device=dev_index)
    res = {}
    raw = fec.host_alloc(2 * n * 1488)
    try:
        rng = np.random.default_rng(args.seed + 5)

        def median_us(call, reps=2000):
            for _ in range(200):
                assert call() == 0
            ts = np.empty(reps)
            for i in range(reps):
                t0 = time.perf_counter_ns()
                call()
                ts[i] = time.perf_counter_ns() - t0
            return round(float(np.median(ts)) / 1e3, 2)

        mask = np.array([((1 << n) - 1) & ~(1 << 3)], np.uint64)
        status = np.zeros(1, np.int8)
        mp = ctypes.c_void_p(mask.ctypes.data)
        sp = ctypes.c_void_p(status.ctypes.data)
        src = {S: rng.integers(0, 256, (1, n, (S + 15) // 16 * 16), dtype=np.uint8) for S in (1470, 1476)}
        outs = {}
        for mode in ("launch", "service"):
            if mode == "service":
                enc.service_start()
            row = {}
            # Encode: the 1470-B calcECC window, parity rows zeroed first
            S, P = 1470, 1472
            g = raw[: n * P].reshape(1, n, P)
            g[:] = src[S]
            g[0, d:, :S] = 0
            ptr = ctypes.c_void_p(g.ctypes.data)
            row["encode_1470_us"] = median_us(lambda: lib.ugo_fec_encode_host(enc._h, ptr, 1, S, P))
            enc_out = g.copy()
            # Reconstruct: a 1476-B codeword with data shard 3 lost
            S2, P2 = 1476, 1488
            g2 = raw[n * 1488: n * 1488 + n * P2].reshape(1, n, P2)
            g2[:] = src[S2]
            ptr2 = ctypes.c_void_p(g2.ctypes.data)
            assert lib.ugo_fec_encode_host(enc._h, ptr2, 1, S2, P2) == 0
            want = g2[0, 3, :S2].copy()
            g2[0, 3, :S2] = 0xEE
            row["reconstruct_1476_1loss_us"] = median_us(
                lambda: lib.ugo_fec_reconstruct_host(enc._h, ptr2, mp, 1, S2, P2, 0, sp))
            row["rebuilt_ok"] = bool(np.array_equal(g2[0, 3, :S2], want))
            outs[mode] = (enc_out, g2.copy())
            res[mode] = row
        enc.service_stop()
        res["service"]["same_bytes_as_launch"] = all(
            bool(np.array_equal(x, y)) for x, y in zip(outs["launch"], outs["service"]))
        try:  # a secondary measurement: a failure is reported, never loses the leg
            res["interference"] = service_interference(args, dev_index, enc, raw)
        except Exception as ex:  # noqa: BLE001
            res["interference"] = {"error": repr(ex)[:300]}
    finally:
        enc.service_stop()
        fec.host_free(raw)
        enc.close()
    res["note"] = ("one (10+3) group per call through the C-ABI from Python (ctypes), the cgo shim's staging: "
                   "launch = one kernel launch + stream synchronize per call; service = ugo_fec_service_start "
                   "(a resident workgroup polls a pinned mailbox); cpu_one_core_us: the same calls on one core of "
                   "this host (cpu_baseline.single_core)")
    return res


def service_interference(args, dev_index, enc, raw, rounds=3, steps=20):
    """What a resident per-call service block (one CU held, a PCIe poll of its
    pinned mailbox) costs concurrent batch work on the same GPU: the bench step
    (encode + reconstruct_into of 65,536 (10+3) groups, 2 cold planar batches)
    and the (10+3) x 65,536 pinned-host encode (PCIe-inclusive, launch path),
    each timed `rounds` times alternately without and with the service
    resident (started with a 1-s idle window and one served call just before
    the timed work); medians.  Timing uses a dedicated stream and its events
    (a device-wide synchronize would wait for the resident block)."""
    import numpy as np
    import torch

    from ugo_amd import fec

    d, p, S, G = 10, 3, 1350, 65536
    n, pitch = d + p, 1360
    dev = torch.device("cuda", dev_index)
    s = torch.cuda.Stream(device=dev)
    gen = torch.Generator(device=dev).manual_seed(args.seed + 0x1F)
    work = fec.New(d, p, device=dev_index)
    bats = [torch.randint(0, 256, (n, G, pitch), dtype=torch.uint8, device=dev, generator=gen) for _ in range(2)]
    outs = [torch.empty((p, G, pitch), dtype=torch.uint8, device=dev) for _ in range(2)]
    masks, _ = make_masks(G, n, 2, args.seed + 0x2F, dev)
    hraw = fec.host_alloc(G * n * pitch)
    hbuf = hraw.reshape(G, n, pitch)
    hbuf[:] = 7
    one = raw[: n * 1472].reshape(1, n, 1472)
    torch.cuda.synchronize()
    try:
        def step_ms():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            with torch.cuda.stream(s):
                for k in range(4):  # warm
                    work.encode_batch(bats[k % 2], shard_size=S, stream=s, shard_major=True)
                    work.reconstruct_into(bats[k % 2], masks, outs[k % 2], shard_size=S, stream=s, shard_major=True)
                e0.record(s)
                for k in range(steps):
                    work.encode_batch(bats[k % 2], shard_size=S, stream=s, shard_major=True)
                    work.reconstruct_into(bats[k % 2], masks, outs[k % 2], shard_size=S, stream=s, shard_major=True)
                e1.record(s)
            e1.synchronize()
            return e0.elapsed_time(e1) / steps

        def host_ms():
            t0 = time.perf_counter()
            work.encode_host(hbuf, S)
            return (time.perf_counter() - t0) * 1e3

        rows = {"off": {"step": [], "host": []}, "on": {"step": [], "host": []}}
        for _ in range(rounds):
            for mode in ("off", "on"):
                if mode == "on":
                    enc.service_start(idle_us=1_000_000)
                    assert enc.encode_host(one, 1470) is None  # served: the block is now resident
                rows[mode]["step"].append(step_ms())
                rows[mode]["host"].append(host_ms())
                if mode == "on":
                    enc.service_stop()
        med = {m: {k: float(np.median(v)) for k, v in r.items()} for m, r in rows.items()}
        return {"step_ms_without": round(med["off"]["step"], 4), "step_ms_with_service": round(med["on"]["step"], 4),
                "step_slowdown": round(med["on"]["step"] / med["off"]["step"] - 1, 4),
                "host_encode_ms_without": round(med["off"]["host"], 3),
                "host_encode_ms_with_service": round(med["on"]["host"], 3),
                "host_encode_slowdown": round(med["on"]["host"] / med["off"]["host"] - 1, 4),
                "rounds": rounds, "steps": steps,
                "note": "service started with a 1-s idle window and one served call before each 'with' sample, "
                        "so its block is resident (polling) through the sample"}
    finally:
        fec.host_free(hraw)
        work.close()


def probe_library():
    """libugoprobe.so: the measurement kernels (ugo_amd/csrc/probe_kernels.hip)
    behind the ceilings -- a separate library the product path never loads."""
    import ctypes

    path = os.path.join(ROOT, "ugo_amd", "libugoprobe.so")
    if not os.path.exists(path):
        raise ImportError(f"{path} not built: run `make -C ugo_amd/csrc`")
    lib = ctypes.CDLL(path)
    vp, sz, i = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
    lib.ugo_probe_encode_twin.argtypes = [vp, i, sz, sz, sz, sz, i, vp, vp]
    lib.ugo_probe_nt_copy.argtypes = [vp, vp, i, sz, i, vp, vp]
    lib.ugo_probe_reconstruct_twin.argtypes = [vp, vp, i, vp, sz, sz, sz, sz, sz, sz, i, vp, vp]
    lib.ugo_probe_recover_twin.argtypes = [vp, vp, vp, vp, vp, i, sz, sz, sz, sz, sz, sz, i, ctypes.c_uint32, i, vp,
                                           vp]
    lib.ugo_probe_pcie.argtypes = [vp, vp, vp, vp, sz, i, vp]
    return lib


def probe_recover_twin_ms(bases, outs, presents, lists, counts, G, S, pitch, rs, ors, oes, reps, stream):
    """Average duration of the RX-path recovery's compute-free twin
    (k_recover_twin, libugoprobe): data only, the full grid (lists None) or the
    list form; launch r on buffer set r % n."""
    import ctypes

    import numpy as np

    lib = probe_library()
    nb = len(bases)
    arr = lambda xs: (ctypes.c_void_p * nb)(*[x.data_ptr() for x in xs])  # noqa: E731
    ms = np.zeros(reps, np.float32)
    rc = lib.ugo_probe_recover_twin(arr(bases), arr(outs), arr(presents), None if lists is None else arr(lists),
                                    None if counts is None else arr(counts), nb, G, S, pitch, rs, ors, oes, 1,
                                    36 * 1024, reps, stream, ms.ctypes.data)
    if rc:
        raise RuntimeError(f"ugo_probe_recover_twin failed ({rc})")
    return float(ms[1:].mean()) if reps > 1 else float(ms[0])


def probe_nt_copy_ms(srcs, dsts, nbytes, reps, stream):
    """Average duration of `reps` nt copies of nbytes (srcs[r % n] -> dsts[r % n],
    device pointers), each launch timed by its own start/stop events."""
    import ctypes

    import numpy as np

    lib = probe_library()
    nb = len(srcs)
    assert nbytes > 0
    S = (ctypes.c_void_p * nb)(*srcs)
    D = (ctypes.c_void_p * nb)(*dsts)
    ms = np.zeros(reps, np.float32)
    rc = lib.ugo_probe_nt_copy(S, D, nb, nbytes // 16 * 16, reps, stream, ms.ctypes.data)
    if rc:
        raise RuntimeError(f"ugo_probe_nt_copy failed ({rc})")
    return float(ms[1:].mean()) if reps > 1 else float(ms[0])


def ceilings(args, batches, G, S, pitch, enc_bytes, stream, masks=None, outs=None, dec_bytes=0):
    """the encode's ceiling measured in this run, on the
    same cold rotated batches (launch r on batch r % B): the compute-free twin
    of k_encode_g (same loads, LDS stage, residency and nt stores; XOR instead
    of the GF network) and a plain nt copy moving the same 1.15 GB (half a
    batch read, the other half written).  Each launch timed with its own
    hipExtLaunchKernel start/stop events, as the kernel pass times the encode.
    With masks and outs (the step's reconstruct into separate outputs): the
    compute-free twin of k_apply_p too, on the same batches and outputs.
    The twins write wrong bytes on purpose: run after the verification."""
    import ctypes

    import numpy as np

    lib = probe_library()
    reps = max(8, min(args.steps, 40))
    nb = len(batches)
    bases = (ctypes.c_void_p * nb)(*[b.data_ptr() for b in batches])
    ms = np.zeros(reps, np.float32)
    rs = batches[0].stride(0)  # planar: bytes between row streams
    rc = lib.ugo_probe_encode_twin(bases, nb, G, S, pitch, rs, reps, stream.cuda_stream, ms.ctypes.data)
    if rc:
        raise RuntimeError(f"ugo_probe_encode_twin failed ({rc})")
    twin_ms = float(ms[1:].mean())
    half = (batches[0].numel() // 2) // 16 * 16
    copy_bytes = enc_bytes // 2 // 16 * 16  # read + written = the encode's algorithmic bytes
    assert copy_bytes <= half
    copy_ms = probe_nt_copy_ms([b.data_ptr() for b in batches], [b.data_ptr() + half for b in batches], copy_bytes,
                               reps, stream.cuda_stream)
    res = {"encode_twin_ms": round(twin_ms, 5), "encode_twin_GBps": round(enc_bytes / (twin_ms * 1e-3) / 1e9, 1),
           "nt_copy_ms": round(copy_ms, 5), "nt_copy_GBps": round(2 * copy_bytes / (copy_ms * 1e-3) / 1e9, 1),
           "reps": reps}
    if masks is not None and outs is not None and dec_bytes:
        ob = (ctypes.c_void_p * nb)(*[o.data_ptr() for o in outs])
        rc = lib.ugo_probe_reconstruct_twin(bases, ob, nb, masks.data_ptr(), G, S, pitch, rs, outs[0].stride(0),
                                            outs[0].stride(1), reps, stream.cuda_stream, ms.ctypes.data)
        if rc:
            raise RuntimeError(f"ugo_probe_reconstruct_twin failed ({rc})")
        rt_ms = float(ms[1:].mean())
        res["reconstruct_twin_ms"] = round(rt_ms, 5)
        res["reconstruct_twin_GBps"] = round(dec_bytes / (rt_ms * 1e-3) / 1e9, 1)
    return res


def rc4_pad(nbytes, dev):
    import torch

    from ugo_amd import fec

    return torch.frombuffer(bytearray(fec.rc4_keystream(b"1234567890123456", nbytes)), dtype=torch.uint8).to(dev)


def lost_and_recoverable(pm, d, n):
    """Per presence mask: erased data rows, and whether >= d of the n rows are present."""
    import torch

    ed = torch.zeros(pm.shape, dtype=torch.int64, device=pm.device)
    have = torch.zeros(pm.shape, dtype=torch.int64, device=pm.device)
    for r in range(n):
        bit = (pm >> r) & 1
        have += bit
        if r < d:
            ed += bit == 0
    return ed, have >= d


RX_LAYOUTS = {  # W = bytes a row carries, off = the payload's column (include/ugo_fec.h)
    "payload": {"frames": False, "W": 1470, "pitch": 1472, "off": 0,
                "rows": "[13][G][1472], the payload realigned to column 0 (ugo_fec_rx_assemble)"},
    "frames": {"frames": True, "W": 1476, "pitch": 1536, "off": 6,
               "rows": "[13][G][1536], each row the decrypted packet, payload at column 6 (ugo_fec_rx_assemble_frames)"},
}
RX_PRIMARY = "frames"  # ahead in 2 of 3 final-tree runs; the other layout is timed beside it


def alt_layout_case(enc, rings, lens, pad, flats, ppres, plsts, pcnts, plouts, G, n, p, S, L, P, kernel_ms, reps,
                    rx_ms):
    """The RX ring into the other layout L (views of the primary batches'
    flat storage, overwritten) and its list recovery: checked equal to the
    primary layout P's presence masks, lossy list and recovered payload columns
    (ppres / plsts / pcnts / plouts of the primary run on rings[0]), then its
    recovery timed (its placement time, rx_ms, comes from the caller's
    alternating rounds).  Placement time depends on which physical pages back a
    batch (up to 15 % between allocations of one process, tools/rx_frames_ab.py
    same), so both layouts are timed on the same pages."""
    import torch

    from ugo_amd import fec

    dev = rings[0].device
    bats = [f[:n * G * L["pitch"]].view(n, G, L["pitch"]) for f in flats]
    pres = [torch.zeros(G, dtype=torch.int64, device=dev) for _ in range(2)]
    lsts = [torch.empty(G, dtype=torch.int32, device=dev) for _ in range(2)]
    cnts = [torch.empty(1, dtype=torch.int32, device=dev) for _ in range(2)]
    outs = [torch.empty((G, p, L["pitch"]), dtype=torch.uint8, device=dev) for _ in range(2)]

    def rx(r):
        i = r % 2
        pres[i].zero_()
        enc.rx_assemble(rings[i], lens, bats[i], pres[i], shard_size=S, pad=pad, frames=L["frames"])

    def rec_list(r):
        i = r % 2
        enc.lossy_groups(pres[i], data_only=True, out=lsts[i], count=cnts[i])
        enc.reconstruct_list(bats[i], pres[i], lsts[i], cnts[i], outs[i], shard_size=L["W"], data_only=True)

    for r in range(4):
        rx(r)
        rec_list(r)
    torch.cuda.synchronize()
    k = int(cnts[0].item())
    ok = k == int(pcnts[0].item()) and bool(torch.equal(pres[0], ppres[0])) and bool(
        torch.equal(lsts[0][:k], plsts[0][:k]))
    if ok:  # each entry's recovered rows (slots past its erasure count are not written by either)
        ed, okg = lost_and_recoverable(pres[0][lsts[0][:k].long()], n - p, n)
        for i in range(p):
            sel = (ed > i) & okg
            ok = ok and bool(torch.equal(outs[0][:k][sel, i, L["off"]:L["off"] + S],
                                         plouts[0][:k][sel, i, P["off"]:P["off"] + S]))
    rec_k = kernel_ms(rec_list, fec.KERNEL_IDS["reconstruct"], reps)
    return {"rows": L["rows"], "rx_assemble_ms": round(rx_ms, 4), "reconstruct_list_ms": round(rec_k, 4),
            "verify_eq_primary": ok,
            "timing": "rx_assemble_ms: the median of 4 rounds alternating with the primary layout's on the same storage"}


def rx_tx_leg(args, dev_index, reps=12):
    """The §8f kernels on the driver's clock, on every rank
    (rank 0 reports its own leg plus the max over ranks of
    each kernel time), after the main line (nothing here feeds `value`).
    Device-resident, cold: every call alternates between 2 copies of its
    inputs and outputs.
      * rx_assemble (ugo/conn.go:387-406 decrypt, ugo/fec.go:78-89 decode,
        :107-175 grouping / dedupe / placement): a ring of 65,536 (10+3) groups
        minus 5% uniform loss, 1476-B packets in 1488-B slots, RC4, into a
        planar batch in the RX_PRIMARY layout (frame rows [13][G][1536], each
        row the decrypted packet, payload at column 6, recovered on the 1476-B
        frame window), with the other layout (payload rows [13][G][1472], the
        payload realigned to column 0, as the host RX path builds them) timed
        beside it on the same storage (`alt_layout`); arrival in
        seqid order (what a UDP flow mostly delivers) and shuffled (worst
        case);
      * reconstruct_into, data only, of the lossy groups of that batch
        (input's Reconstruct, ugo/fec.go:196-207), over every group, and its
        list form (lossy_groups + reconstruct_list: only the lossy groups,
        compact outputs), each beside its compute-free twin (the same loads
        and stores, XOR instead of the GF products) on the same buffers;
      * tx_assemble (ugo/conn.go:643-685 sender loop + :634 encrypt): 65,536
        groups of 10 full 1476-B packets -> 13 wire packets each, RC4;
      * packet_decode (ugo/packet.go:138-177 after conn.go:387-419): 851,968
        FEC-framed RC4 packets, one segment, a quarter with a SACK.
    Kernel times from hipExtLaunchKernel events (every launch of the call),
    bytes: RX packet bytes read + payload written; TX data packets read + wire
    packets written; reconstruct d survivor rows read + e data rows written per
    lossy group.  Next to each, an nt copy moving the same bytes in this
    process (libugoprobe): the copy ceiling."""
    import numpy as np
    import torch

    from ugo_amd import fec

    d, p, n, S, slot = 10, 3, 13, 1470, 1488
    PL = RX_LAYOUTS[RX_PRIMARY]
    alt = [k for k in RX_LAYOUTS if k != RX_PRIMARY][0]
    AL = RX_LAYOUTS[alt]
    W, pitch, off = PL["W"], PL["pitch"], PL["off"]
    span = max(L["pitch"] for L in RX_LAYOUTS.values())  # storage per row for either layout's view
    G = 65536
    dev = torch.device("cuda", dev_index)
    stream = torch.cuda.current_stream(dev)
    enc = fec.New(d, p, device=dev_index)
    pad = rc4_pad(slot, dev)
    gen = torch.Generator(device=dev).manual_seed(args.seed + 0x5A)
    out = {}

    def kernel_ms(fn, kid, calls):
        enc.timing_begin(16 * calls)
        for r in range(calls):
            fn(r)
        recs, _ = enc.timing_end()
        ids = kid if isinstance(kid, tuple) else (kid,)
        return float(recs["ms"][np.isin(recs["kernel"], ids)].sum()) / calls

    def wall_ms(fn, calls):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record(stream)
        for r in range(calls):
            fn(r)
        e1.record(stream)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / calls

    def frac(b, ms):
        return round(b / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)

    # ---- RX + data-only recovery
    seq_all = torch.arange(G * n, device=dev, dtype=torch.int64)
    keep = torch.rand(G * n, device=dev, generator=gen) >= 0.05
    for order in ("in_order", "shuffled"):
        seq = seq_all[keep]
        if order == "shuffled":
            seq = seq[torch.randperm(seq.numel(), device=dev, generator=gen)]
        npk = seq.numel()
        rings = []
        for _ in range(2):
            w = torch.randint(0, 256, (npk, slot), dtype=torch.uint8, device=dev, generator=gen)
            hdr = torch.zeros((npk, 6), dtype=torch.uint8, device=dev)
            for b in range(4):
                hdr[:, b] = ((seq >> (8 * b)) & 0xFF).to(torch.uint8)
            hdr[:, 4] = torch.where(seq % n < d, 0xF1, 0xF2).to(torch.uint8)
            w[:, :6] = hdr ^ pad[:6]
            rings.append(w)
        lens = torch.full((npk,), 1476, dtype=torch.int16, device=dev)
        flats = [torch.empty(n * G * span, dtype=torch.uint8, device=dev) for _ in range(2)]  # either layout's view
        bats = [f[:n * G * pitch].view(n, G, pitch) for f in flats]
        pres = [torch.zeros(G, dtype=torch.int64, device=dev) for _ in range(2)]
        outs = [torch.empty((p, G, pitch), dtype=torch.uint8, device=dev) for _ in range(2)]
        st = torch.zeros(5, dtype=torch.int32, device=dev)

        def rx(r):
            i = r % 2
            pres[i].zero_()
            enc.rx_assemble(rings[i], lens, bats[i], pres[i], shard_size=S, pad=pad, stats=st, frames=PL["frames"])

        def rec(r):
            i = r % 2
            enc.reconstruct_into(bats[i], pres[i], outs[i], shard_size=W, data_only=True, shard_major=True)

        for r in range(4):
            rx(r)
            rec(r)
        st.zero_()
        rx(0)
        torch.cuda.synchronize()
        stats = st.tolist()
        # spot check of the placement: 4,096 packets' payloads, decrypted, in their rows
        pick = torch.randint(0, npk, (4096,), device=dev, generator=gen)
        sq = seq[pick]
        want = rings[0][pick, 6 - off:6 - off + W] ^ pad[6 - off:6 - off + W]
        got = bats[0][sq % n, sq // n, :W]
        ok = stats == [npk, 0, 0, 0, 0] and bool(torch.equal(got, want))
        # both layouts timed alternately, on the same storage (placement time moves with the physical pages
        # a batch gets): the median of 4 rounds each
        abats = [f[:n * G * AL["pitch"]].view(n, G, AL["pitch"]) for f in flats]
        apres = [torch.zeros(G, dtype=torch.int64, device=dev) for _ in range(2)]

        def arx(r):
            i = r % 2
            apres[i].zero_()
            enc.rx_assemble(rings[i], lens, abats[i], apres[i], shard_size=S, pad=pad, frames=AL["frames"])

        tp, ta = [], []
        for rnd in range(4):
            for fn, acc in (((rx, tp), (arx, ta)) if rnd % 2 == 0 else ((arx, ta), (rx, tp))):
                fn(0)
                fn(1)
                acc.append(kernel_ms(fn, fec.KERNEL_IDS["rx_assemble"], reps))
        rx_k, arx_k = float(np.median(tp)), float(np.median(ta))
        del abats, apres
        for r in range(2):  # the primary rows back for the recovery below
            rx(r)
        rx_w = wall_ms(rx, reps)
        rec_k = kernel_ms(rec, (fec.KERNEL_IDS["reconstruct"], fec.KERNEL_IDS["prepare"]), reps)
        m = pres[0].cpu().numpy().view(np.uint64)
        lost_data = np.zeros(G, np.int64)
        for r in range(d):
            lost_data += ((m >> np.uint64(r)) & np.uint64(1)) == 0
        pop = np.zeros(G, np.int64)
        for r in range(n):
            pop += ((m >> np.uint64(r)) & np.uint64(1)).astype(np.int64)
        recoverable = (lost_data > 0) & (pop >= d)
        rec_bytes = int((recoverable * (d + lost_data)).sum()) * S
        rx_bytes = npk * (1476 + S)
        # the list form: lossy-group list + list reconstruct, compact outputs
        lsts = [torch.empty(G, dtype=torch.int32, device=dev) for _ in range(2)]
        cnts = [torch.empty(1, dtype=torch.int32, device=dev) for _ in range(2)]
        louts = [torch.empty((G, p, pitch), dtype=torch.uint8, device=dev) for _ in range(2)]

        def rec_list(r):
            i = r % 2
            enc.lossy_groups(pres[i], data_only=True, out=lsts[i], count=cnts[i])
            enc.reconstruct_list(bats[i], pres[i], lsts[i], cnts[i], louts[i], shard_size=W, data_only=True)

        for r in range(4):
            rx(r)
            rec(r)
            rec_list(r)
        torch.cuda.synchronize()
        # the two forms agree: entry j's slot i = group lst[j]'s output i of reconstruct_into
        k = int(cnts[0].item())
        lg = lsts[0][:k].long()
        ed, okg = lost_and_recoverable(pres[0][lg], d, n)
        ok_list = k == int((lost_data > 0).sum())
        for i in range(p):
            sel = (ed > i) & okg  # groups below d shards: no output in either form
            ok_list = ok_list and bool(torch.equal(louts[0][:k][sel, i, off:off + S],
                                                   outs[0][i, lg[sel], off:off + S]))
        rec_list_k = kernel_ms(rec_list, fec.KERNEL_IDS["reconstruct"], reps)
        # the same recovery as `input` returns it (ugo_fec_recover_data): the lost data shards
        # row-compact in `recovered` order with their places, the count on the device
        rdo = [torch.empty((G * min(d, p), pitch), dtype=torch.uint8, device=dev) for _ in range(2)]
        rdi = [torch.empty(G * min(d, p), dtype=torch.int32, device=dev) for _ in range(2)]
        rdc = [torch.empty(1, dtype=torch.int32, device=dev) for _ in range(2)]

        def rec_data(r):
            i = r % 2
            enc.recover_data(bats[i], pres[i], rdo[i], rdi[i], count=rdc[i], shard_size=W)

        for r in range(2):
            rx(r)
            rec_data(r)
        torch.cuda.synchronize()
        nr = int(rdc[0].item())
        lost = ((pres[0][lg][:, None] >> torch.arange(d, device=dev)) & 1) == 0
        lost &= okg[:, None]
        jj, rr = torch.nonzero(lost, as_tuple=True)
        want_rows = louts[0][:k][torch.arange(p, device=dev)[None, :] < lost.sum(1)[:, None]]
        ok_rd = nr == int(jj.numel()) and bool(torch.equal(rdi[0][:nr].long(), lg[jj] * n + rr)) and bool(
            torch.equal(rdo[0][:nr, off:off + S], want_rows[:, off:off + S]))
        rec_data_k = kernel_ms(rec_data, fec.KERNEL_IDS["reconstruct"], reps)
        del rdo, rdi, rdc
        # the other layout on the same rings and storage, checked against the primary one, with its recovery
        al = alt_layout_case(enc, rings, lens, pad, flats, pres, lsts, cnts, louts, G, n, p, S, AL, PL, kernel_ms,
                             reps, arx_k)
        # ceilings: the compute-free twins of both forms on the same buffers (after the checks: wrong bytes)
        twin_ms = probe_recover_twin_ms(bats, outs, pres, None, None, G, W, pitch, bats[0].stride(0),
                                        outs[0].stride(0), outs[0].stride(1), reps, stream.cuda_stream)
        ltwin_ms = probe_recover_twin_ms(bats, louts, pres, lsts, cnts, G, W, pitch, bats[0].stride(0),
                                         louts[0].stride(1), louts[0].stride(0), reps, stream.cuda_stream)
        cb = min(rx_bytes // 2, rings[0].numel(), bats[0].numel())  # each copy stays inside both buffers
        copy_ms = probe_nt_copy_ms([rings[i].data_ptr() for i in range(2)], [bats[(i + 1) % 2].data_ptr()
                                                                            for i in range(2)],
                                   cb, reps, stream.cuda_stream) * (rx_bytes // 2) / cb
        out[f"rx_{order}"] = {
            "packets": npk, "groups": G, "loss": 0.05, "rc4": True,
            "rx_assemble_ms": round(rx_k, 4), "rx_assemble_wall_ms": round(rx_w, 4),
            "rx_GBps": round(rx_bytes / (rx_k * 1e-3) / 1e9, 1), "rx_frac": frac(rx_bytes, rx_k),
            "rx_Mpkt_per_s": round(npk / (rx_k * 1e-3) / 1e6, 1),
            "nt_copy_same_bytes_ms": round(copy_ms, 4), "nt_copy_frac": frac(rx_bytes, copy_ms),
            "rx_frac_of_copy": round(copy_ms / rx_k, 4),
            "recover_lossy_groups": int(recoverable.sum()), "reconstruct_into_data_only_ms": round(rec_k, 4),
            "reconstruct_GBps": round(rec_bytes / (rec_k * 1e-3) / 1e9, 1), "reconstruct_frac": frac(rec_bytes, rec_k),
            "reconstruct_twin_ms": round(twin_ms, 4), "reconstruct_frac_of_ceiling": round(twin_ms / rec_k, 4),
            "reconstruct_list_ms": round(rec_list_k, 4), "reconstruct_list_frac": frac(rec_bytes, rec_list_k),
            "reconstruct_list_twin_ms": round(ltwin_ms, 4),
            "reconstruct_list_frac_of_ceiling": round(ltwin_ms / rec_list_k, 4),
            "recovery_faster": "list" if rec_list_k < rec_k else "into", "verify_list_eq_into": ok_list,
            "recover_data_ms": round(rec_data_k, 4), "recover_data_frac": frac(rec_bytes, rec_data_k),
            "verify_recover_data": ok_rd,
            "stats": stats, "verify_spot_4096": ok,
            "layout": f"{RX_PRIMARY}: {PL['rows']}",
            "rx_rounds_ms": {RX_PRIMARY: [round(x, 4) for x in tp], alt: [round(x, 4) for x in ta],
                             "note": f"alternating rounds on the same storage; rx_assemble_ms = median of {RX_PRIMARY}"},
            "alt_layout": {"name": alt, **al, "rx_frac": frac(rx_bytes, al["rx_assemble_ms"]),
                           "reconstruct_list_frac": frac(rec_bytes, al["reconstruct_list_ms"])}}
        del rings, bats, flats, pres, outs, lsts, cnts, louts
        torch.cuda.empty_cache()

    # ---- TX
    max_len = 1476
    pks = [torch.randint(0, 256, (G * d, slot), dtype=torch.uint8, device=dev, generator=gen) for _ in range(2)]
    tl = torch.full((G * d,), max_len, dtype=torch.int16, device=dev)
    wires = [torch.empty((G * n, slot), dtype=torch.uint8, device=dev) for _ in range(2)]
    wls = [torch.empty(G * n, dtype=torch.int16, device=dev) for _ in range(2)]

    def tx(r):
        i = r % 2
        enc.tx_assemble(pks[i], tl, wires[i], wls[i], pad=pad, max_len=max_len)

    for r in range(4):
        tx(r)
    torch.cuda.synchronize()
    # spot check: data packet k of group g on the wire = header + payload, encrypted
    g = 12345
    w0 = (wires[1][g * n: g * n + d, :max_len] ^ pad[:max_len])
    ok_tx = bool(torch.equal(w0[:, 6:], pks[1][g * d: g * d + d, 6:max_len])) and bool(
        (wls[1][g * n: g * n + n] == max_len).all())
    tx_k = kernel_ms(tx, fec.KERNEL_IDS["tx_assemble"], reps)
    tx_bytes = G * (d + n) * max_len
    # wire buffers on both sides: the data packets alone (G*d*slot) hold fewer bytes than half the bytes moved
    cb = min(tx_bytes // 2, wires[0].numel())
    copy_ms = probe_nt_copy_ms([wires[i].data_ptr() for i in range(2)], [wires[(i + 1) % 2].data_ptr()
                                                                         for i in range(2)],
                               cb, reps, stream.cuda_stream) * (tx_bytes // 2) / cb
    out["tx"] = {"groups": G, "packets_out": G * n, "rc4": True, "tx_assemble_ms": round(tx_k, 4),
                 "tx_GBps": round(tx_bytes / (tx_k * 1e-3) / 1e9, 1), "tx_frac": frac(tx_bytes, tx_k),
                 "tx_Mpkt_per_s": round(G * n / (tx_k * 1e-3) / 1e6, 1),
                 "nt_copy_same_bytes_ms": round(copy_ms, 4), "nt_copy_frac": frac(tx_bytes, copy_ms),
                 "tx_frac_of_copy": round(copy_ms / tx_k, 4), "verify_spot": ok_tx}
    del pks, wires, wls
    torch.cuda.empty_cache()

    # ---- packet decode
    out["packet_decode"] = packet_decode_case(enc, dev, reps, kernel_ms)
    out["note"] = ("kernel ms = sum of the call's launches (hipExtLaunchKernel events); frac = algorithmic bytes / "
                   "kernel time / 8 TB/s; nt_copy = libugoprobe's one-chunk-per-thread nt copy moving the same "
                   "bytes on the same cold buffers; rx_wall includes the caller's present.zero_() per call")
    enc.close()
    return out


def rx_tx_over_ranks(mine, legs):
    """Rank 0's rx_tx leg with, for every kernel time of it (keys ending in
    _ms), the max over the ranks' legs (`max_over_ranks`) and each rank's
    value (`per_rank`)."""
    def times(d, pre=""):
        out = {}
        for k, v in (d or {}).items():
            if isinstance(v, dict):
                out.update(times(v, pre + k + "."))
            elif k.endswith("_ms") and isinstance(v, (int, float)):
                out[pre + k] = v
        return out

    per = [times(x) for x in legs]
    keys = sorted(set().union(*per)) if per else []
    res = dict(mine)
    res["max_over_ranks"] = {k: max(t.get(k, 0.0) for t in per) for k in keys}
    res["per_rank"] = [{k: t.get(k) for k in keys} for t in per]
    res["ranks"] = len(legs)
    return res


def packet_decode_case(enc, dev, reps, kernel_ms, npk=851968):
    """ugo_fec_packet_decode over npk received packets: FEC-framed, RC4, flags
    PSH (a quarter with a SACK frame), 3-byte packet number, one 1400-B segment."""
    import numpy as np
    import torch

    from ugo_amd import fec

    slot = 1488
    rng = np.random.default_rng(11)
    host = rng.integers(0, 256, (npk, slot), dtype=np.uint8)
    seqn = np.arange(npk, dtype=np.uint64)
    host[:, 0:4] = seqn.astype("<u4").view(np.uint8).reshape(npk, 4)
    host[:, 4] = 0xF1
    host[:, 5] = 0

    def uvarint(v, nbytes):
        o = np.zeros((v.size, nbytes), np.uint8)
        for j in range(nbytes):
            o[:, j] = ((v >> np.uint64(7 * j)) & np.uint64(0x7F)).astype(np.uint8)
            if j < nbytes - 1:
                o[:, j] |= 0x80
        return o

    ack = rng.random(npk) < 0.25
    pos = np.full(npk, 7)
    host[:, 6] = np.where(ack, 0xA0, 0x20)
    sack = np.concatenate([np.zeros((npk, 1), np.uint8), uvarint(seqn + np.uint64(1 << 15), 3),
                           np.full((npk, 2), 7, np.uint8), np.full((npk, 1), 5, np.uint8)], axis=1)
    rows = np.nonzero(ack)[0]
    host[rows[:, None], 7 + np.arange(7)[None, :]] = sack[rows]
    pos[ack] += 7
    hdr = np.concatenate([uvarint(seqn + np.uint64(1 << 15), 3), uvarint(seqn * np.uint64(1400), 4),
                          np.tile(np.array([[1400 >> 8, 1400 & 0xFF]], np.uint8), (npk, 1))], axis=1)
    for j in range(9):
        host[np.arange(npk), pos + j] = hdr[:, j]
    lens = (pos + 9 + 1400).astype(np.int16)
    ks = np.frombuffer(fec.rc4_keystream(b"1234567890123456", slot), np.uint8)
    host ^= ks[None, :]
    d_pk = torch.from_numpy(host).to(dev)
    d_len = torch.from_numpy(lens).to(dev)
    pad = torch.from_numpy(ks.copy()).to(dev)
    bufs = enc.packet_decode(d_pk, d_len, pad=pad, framed=True, max_ranges=4, max_segments=2)
    torch.cuda.synchronize()
    info = bufs[0].cpu().numpy().view(fec.PKT_INFO_DTYPE).reshape(-1)
    ok = bool((info["status"] == 0).all() and (info["n_segments"] == 1).all())

    def run(_r):
        enc.packet_decode(d_pk, d_len, pad=pad, framed=True, max_ranges=4, max_segments=2, out=bufs)

    for r in range(3):
        run(r)
    ms = kernel_ms(run, fec.KERNEL_IDS["packet_decode"], reps)
    return {"packets": npk, "packet_decode_ms": round(ms, 4), "Mpkt_per_s": round(npk / (ms * 1e-3) / 1e6, 1),
            "bound": "latency (one thread per packet parses ~64 B; segment data is located, not read)",
            "verify_all_decode": ok}


def run_rank(args):
    import numpy as np
    import torch

    from ugo_amd import fec

    rank, local_rank, world = dist_setup(args.dist_backend)
    if world != args.gpus and "WORLD_SIZE" in os.environ:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started {world} ranks")
    ndev = torch.cuda.device_count()
    if ndev < 1:
        raise SystemExit("bench.py: no GPU visible (the product path has no CPU fallback)")
    dev_index = local_rank % ndev
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    ranks_per_device = -(-world // ndev) if world > ndev else 1
    d, p, S = args.data_shards, args.parity_shards, args.shard_size
    n = d + p
    pitch = args.pitch or (S + 15) // 16 * 16
    g0, G, scaling, total_groups = rank_groups(args.total_groups, args.groups, rank, world)
    e = args.erasures

    enc = fec.New(d, p, device=dev_index)
    gen = torch.Generator(device=dev).manual_seed(args.seed + g0)
    planar = args.layout == "planar"
    shape = (n, G, pitch) if planar else (G, n, pitch)
    nb = max(1, args.batches)
    def new_batch():
        if not planar or args.row_pad == 0:
            return torch.randint(0, 256, shape, dtype=torch.uint8, device=dev, generator=gen)
        # planar rows args.row_pad bytes further apart than G*pitch: a strided view
        rs = G * pitch + args.row_pad
        flat = torch.randint(0, 256, (n * rs,), dtype=torch.uint8, device=dev, generator=gen)
        return flat.as_strided((n, G, pitch), (rs, pitch, 1))

    batches = [new_batch() for _ in range(nb)]
    shards = batches[0]
    masks, erased = make_masks(G, n, e, args.seed + 1000 + rank, dev)
    into = args.decode == "into"
    # one output batch per input batch, so every step's outputs are cold too
    opitch = args.out_pitch or pitch
    oplanar = args.out_layout == "planar"
    oshape = (p, G, opitch) if oplanar else (G, p, opitch)
    outs = [torch.zeros(oshape, dtype=torch.uint8, device=dev) for _ in range(nb)] if into else None
    stream = torch.cuda.current_stream()
    cur = [0]

    def step():
        i = cur[0] % nb
        b = batches[i]
        cur[0] += 1
        enc.encode_batch(b, shard_size=S, stream=stream, shard_major=planar)
        if into:
            enc.reconstruct_into(b, masks, outs[i], shard_size=S, stream=stream, shard_major=planar,
                                 out_shard_major=oplanar)
        else:
            enc.reconstruct_batch(b, masks, shard_size=S, stream=stream, shard_major=planar)

    sync = torch.cuda.synchronize
    cw_ms, cw_steps, cw_settled = clock_warmup(step, sync, args.clock_warmup_ms)
    barrier(world)  # ranks start the counted warm-up together, none idles after its clock warm-up
    for _ in range(args.warmup):
        step()
    sync()

    # 1. The timed region (`value`): K steps of ordinary launches, barrier +
    #    synchronize on both sides, max over ranks.
    elapsed = timed_region(step, args.steps, sync, world)

    # 2. Kernel-timing pass (`roofline`, `kernels`): the same K steps again with
    #    per-launch start/stop events (kernel_pass); the value pass above runs
    #    without them.
    enc_ms, dec_ms, elapsed_timing_pass = kernel_pass(enc, step, args.steps, sync)

    elapsed, enc_ms_max, dec_ms_max = reduce_max([elapsed, enc_ms, dec_ms], world)

    enc_bytes = G * n * S            # per launch, this rank
    dec_bytes = G * (d + e) * S
    step_bytes_all = total_groups * (n * S + (d + e) * S)
    value = step_bytes_all * args.steps / elapsed / 2**30

    # bit-exactness at full size (outside the timed region): erase, reconstruct, compare
    verify = None
    if not args.no_verify:
        view = shards.transpose(0, 1) if planar else shards  # [G, n, pitch] view either way
        ref = view.clone()
        gi = torch.arange(G, device=dev)
        for j in range(e):
            view[gi, erased[:, j].to(dev)] = 0
        if into:
            o = torch.full((p, G, opitch), 0xA5, dtype=torch.uint8, device=dev)
            enc.reconstruct_into(shards, masks, o, shard_size=S, stream=stream, shard_major=planar)
            es = erased.sort(dim=1).values.to(dev)  # output j = j-th erased row, ascending
            ok_rt = all(bool(torch.equal(o[j, :, :S], ref[gi, es[:, j], :S])) for j in range(e))
            for j in range(e):  # the input keeps its erased (zeroed) rows
                ok_rt = ok_rt and not bool(view[gi, es[:, j], :S].any())
            del o
        else:
            enc.reconstruct_batch(shards, masks, shard_size=S, stream=stream, shard_major=planar)
            ok_rt = bool(torch.equal(view[:, :, :S], ref[:, :, :S]))
        par = ref[:, d:, :S].clone()
        view[:, d:, :] = 0
        enc.encode_batch(shards, shard_size=S, stream=stream, shard_major=planar)
        if into:  # restore the erased data rows so the parity check sees the full data
            view[:, :d, :] = ref[:, :d, :]
            enc.encode_batch(shards, shard_size=S, stream=stream, shard_major=planar)
        ok_idem = bool(torch.equal(view[:, d:, :S], par))
        del ref, par
        verify = {"round_trip_full_size": ok_rt, "encode_idempotent": ok_idem}
        verify["all_ranks_ok"] = all_ranks_ok(ok_rt and ok_idem, world)

    # 2b. Ceilings on the same cold rotated batches (after the verification:
    #     the compute-free twin writes wrong parity on purpose).
    ceil = None
    if planar and args.row_pad == 0 and d == 10 and p == 3 and nb >= 1:
        try:
            oplan = into and oplanar and outs is not None
            ceil = ceilings(args, batches, G, S, pitch, G * n * S, stream, masks if oplan else None,
                            outs if oplan else None, dec_bytes)
        except Exception as ex:  # noqa: BLE001 -- a secondary measurement never loses the line
            ceil = {"error": repr(ex)[:300]}

    # 3. Secondary legs, after the main line's measurement (nothing in them
    #    feeds `value`): BASELINE configs[3] strong over the ranks, and at N = 1
    #    the PCIe-inclusive host path (configs[4] among it).
    #    The host path runs before the 74-GB configs[3] batch is allocated: after
    #    that allocation (freed, cache emptied) the host TX leg's H2D and D2H
    #    copies stopped overlapping for the rest of the process (39 vs 31 ms,
    #    profiles/r5/host_tx_leg_order.txt).
    batches = outs = shards = view = None
    torch.cuda.empty_cache()
    host = None
    if not args.no_host_path:
        try:  # every rank at once, NUMA-local (a secondary leg: failures are reported, never lose the line)
            host = host_path_leg(args, dev_index, rank, world)
        except Exception as ex:  # noqa: BLE001
            host = {"error": repr(ex)[:300]}
    strong = strong_leg(args, enc, rank, world, dev, stream) if args.c4_total_groups > 0 else None
    per_call = rx_tx = None
    if world == 1 and not args.no_host_path:
        try:
            per_call = per_call_leg(args, dev_index)
        except Exception as ex:  # noqa: BLE001
            per_call = {"error": repr(ex)[:300]}
    if not args.no_rx_tx:
        try:  # every rank (device-local work): rank 0's leg plus the max over ranks of each kernel time
            rx_tx = rx_tx_leg(args, dev_index)
        except Exception as ex:  # noqa: BLE001
            rx_tx = {"error": repr(ex)[:300]}
        if world > 1:
            rx_tx = rx_tx_over_ranks(rx_tx, gather_objects(rx_tx, world))

    if rank == 0:
        payload = G * d * S  # klauspost's convention: data bytes per call (BASELINE.md secondary column)
        kern = kernel_stats(enc_ms, dec_ms, enc_bytes, dec_bytes, payload)
        dom = "encode" if enc_ms >= dec_ms else "reconstruct"
        traffic = None
        try:
            tj = json.load(open(args.traffic_json))
            key = f"{dom}:{d}+{p}x{S}/{pitch}:G{G}" + (":into" if into and dom == "reconstruct" else "")
            traffic = tj.get(key)
        except Exception:
            pass
        traffic_note = ("traffic: HBM bytes per launch from the committed rocprofv3 PMC passes "
                        f"({os.path.relpath(args.traffic_json, ROOT)}, (2*FETCH_SIZE + WRITE_SIZE)*1024 per "
                        "MI355X_MICROARCH.md), not counters read in this run") if traffic else None
        ach = kern[dom]["GBps"]
        roof = {"bound": "hbm", "kernel": dom, "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic}
        if ceil and "encode_twin_GBps" in ceil and dom == "encode":
            roof["ceiling_GBps"] = ceil["encode_twin_GBps"]
            roof["frac_of_ceiling"] = round(ach / ceil["encode_twin_GBps"], 4)
            roof["nt_copy_GBps"] = ceil["nt_copy_GBps"]
            roof["ceiling"] = dict(ceil, what=(
                "measured in this run on the same 2 cold rotated batches: encode_twin = k_encode_g's compute-free "
                "twin (same LDS-DMA / register loads, 52-KiB stage = 3 blocks per CU, nt stores; XOR instead of the "
                "GF network), GBps of the encode's algorithmic bytes; nt_copy = a 1-chunk-per-thread nt copy "
                "moving the same 1.15 GB; reconstruct_twin = k_apply_p's compute-free twin (same grid, the first d "
                "present rows of each group by nt loads, one nt store per erased row into the same output batches; "
                "XOR instead of the split-table products), GBps of the reconstruct's algorithmic bytes "
                "(libugoprobe.so, ugo_amd/csrc/probe_kernels.hip)"))
        elif ceil:
            roof["ceiling"] = ceil
        if ceil and "reconstruct_twin_GBps" in ceil and "reconstruct" in kern:
            kern["reconstruct"]["twin_GBps"] = ceil["reconstruct_twin_GBps"]
            kern["reconstruct"]["frac_of_twin"] = round(kern["reconstruct"]["GBps"] / ceil["reconstruct_twin_GBps"], 4)
        roof.update({
                "note": f"achieved = algorithmic bytes per launch ({'(d+p)*S' if dom == 'encode' else '(d+e)*S'}"
                        f" per group x {G} groups) / avg kernel duration over a kernel-timing pass of the same "
                        f"{args.steps} steps right after the timed region, from hipExtLaunchKernel start/stop "
                        f"events on the launch stream (ms_per_step of that pass: "
                        f"{elapsed_timing_pass / args.steps * 1e3:.4f})"
                        + (f"; {traffic_note}" if traffic_note else "")})
        if scaling == "strong":
            workload = f"{total_groups} groups total, strong: {G} groups on rank 0"
        else:
            workload = f"{G} groups/GPU, weak: {total_groups} groups total"
        out = {
            "metric": METRIC, "value": round(value, 3), "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
            "scaling": scaling, "vs_baseline": None, "dtype": "u8",
            "data": "synthetic: device-generated uniform random bytes (seeded), "
                    f"{e} distinct uniformly random erased shards per group",
            "config": {"workload": f"({d}+{p})x{S}B groups, encode + {e}-erasure reconstruct, device-resident, "
                                   + workload, "groups_per_gpu": G, "total_groups": total_groups,
                       "data_shards": d, "parity_shards": p, "shard_size": S, "pitch": pitch, "erasures": e,
                       "layout": "shard-major [d+p][G][pitch]" if planar else "group-major [G][d+p][pitch]",
                       "row_stride": (G * pitch + args.row_pad) if planar else pitch,
                       "batches_per_gpu": nb, "decode": args.decode,
                       "parallelism": f"dp{world} (independent packet groups, no collective)"},
            "clock_warmup_ms": round(cw_ms, 1), "clock_warmup_steps": cw_steps, "clock_settled": cw_settled,
            "untimed_steps_total": cw_steps + args.warmup,
            "pct_hbm_roofline": round(step_bytes_all / world * args.steps / elapsed / (HBM_PEAK_GBS * 1e9), 4),
            "roofline": roof, "kernels": kern, "verify": verify,
        }
        if ranks_per_device > 1:
            out["config"]["ranks_per_device"] = ranks_per_device
            out["note"] = (f"{world} ranks on {ndev} device(s): a launcher rehearsal, not an {world}-GPU "
                           f"measurement")
        if strong is not None:
            out["strong_c4"] = strong
        if host is not None:
            out["host_path"] = host
        if per_call is not None:
            out["per_call"] = per_call
        if rx_tx is not None:
            out["rx_tx"] = rx_tx
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(args, d, p, S, n)
            if per_call is not None and "launch" in per_call:
                sc = out["cpu_baseline"]["single_core"]
                per_call["cpu_one_core_us"] = {"encode": sc["per_group_us"]["encode"],
                                               "reconstruct_1loss": sc["per_group_us"]["reconstruct_1loss"],
                                               "pair_from_steady_rate": sc["pair_us_from_steady_rate"]}
        print(json.dumps(out), flush=True)
    if world > 1:
        import torch.distributed as dist

        dist.destroy_process_group()


def main(argv=None):
    argv = sys.argv[1:] if argv is None else list(argv)
    args = parse(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # nothing here has touched a GPU yet: start the ranks as a child process
        sys.exit(launch(argv, args.gpus))
    run_rank(args)


if __name__ == "__main__":
    main()
