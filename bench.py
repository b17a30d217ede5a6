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
                    help="skip the PCIe-inclusive host_path leg (N = 1): pinned-host encode / reconstruct of "
                         "(10+3)x1350 x 65,536 and (32+8)x9000 x 8,192 groups")
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
        dist.init_process_group(backend, init_method="env://")
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
        v_all, n_all, t_all = leg(c0, 1, args.cpu_baseline_seconds)
        v_one, n_one, t_one = leg(c0[:1], 1, args.cpu_baseline_seconds)
        # per call on 1 core (the drop-in per-group path's CPU figure):
        # the C loop makes one Encode / Reconstruct per group, no ctypes in between
        sh, masks = c0[0]
        per = {"encode": [], "reconstruct_1loss": []}
        for _ in range(20):
            t0 = time.perf_counter()
            rs_ref.c_encode(d, p, sh, threads=1)
            t1 = time.perf_counter()
            rs_ref.c_reconstruct(d, p, sh, masks, threads=1)
            t2 = time.perf_counter()
            per["encode"].append((t1 - t0) / sh.shape[0] * 1e6)
            per["reconstruct_1loss"].append((t2 - t1) / sh.shape[0] * 1e6)
        per_us = {k: round(sorted(v)[len(v) // 2], 3) for k, v in per.items()}
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
                           "seconds": round(t_one, 2), "per_group_us": per_us},
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
    step_bytes = total * (n * S + (d + e) * S)
    res = {"workload": f"BASELINE configs[3]: {total} groups ({d}+{p})x{S}B total, strong over {world} rank(s): "
                       f"{G} groups on rank 0, one cold planar batch per rank, encode + {e}-erasure "
                       f"reconstruct_into",
           "total_groups": total, "groups_per_rank": G, "steps": args.c4_steps, "scaling": "strong",
           "value": round(step_bytes * args.c4_steps / elapsed / 2**30, 3), "unit": "GiB/s",
           "ms_per_step": round(elapsed / args.c4_steps * 1e3, 4),
           "kernels_rank_max": kernel_stats(enc_ms, dec_ms, G * n * S, G * (d + e) * S, G * d * S),
           "verify_round_trip_full_size": ok}
    del sh, out, masks, view
    torch.cuda.empty_cache()
    return res


def host_path_leg(args, dev_index):
    """The PCIe-inclusive rate north_star asks for (the path starts and ends in
    host memory: UDP socket buffers, /root/reference/ugo/conn.go:387-406).
    Batches in pinned host memory (ugo_fec_host_alloc), group-major as a
    packet ring lays them out:
      * (10+3)x1350 x 65,536 groups: ugo_fec_encode_host, then 2 uniformly
        random erasures per group and ugo_fec_reconstruct_host;
      * (32+8)x9000 x 8,192 groups (BASELINE configs[4]): encode, then a
        uniformly random 0..8 erasures per group (mixed patterns) and
        reconstruct.
    The encode stages through device buffers (H2D of the data rows -> kernel
    -> D2H of the parity rows, pipelined over 3 streams); the reconstruct of a
    pinned batch runs zero-copy on its device mapping.  Each
    call: 1 untimed + 3 timed, median.  Verified: every rebuilt batch equals
    the encoded batch it was erased from (compared on the device)."""
    import numpy as np
    import torch

    from ugo_amd import fec

    dev = torch.device("cuda", dev_index)
    res = {}
    for d, p, S, G, mixed in ((10, 3, 1350, 65536, False), (32, 8, 9000, 8192, True)):
        n = d + p
        pitch = (S + 15) // 16 * 16
        enc = fec.New(d, p, device=dev_index)
        raw = fec.host_alloc(G * n * pitch)
        try:
            buf = raw.reshape(G, n, pitch)
            gen = torch.Generator(device=dev).manual_seed(args.seed + d)
            torch.from_numpy(buf).copy_(torch.randint(0, 256, (G, n, pitch), dtype=torch.uint8, device=dev,
                                                      generator=gen))
            times = []
            for k in range(4):
                t0 = time.perf_counter()
                enc.encode_host(buf, S)
                times.append(time.perf_counter() - t0)
            t_enc = sorted(times[1:])[1]
            ref = torch.from_numpy(buf).to(dev)
            rng = np.random.default_rng(args.seed + 7 * d)
            ranks = rng.random((G, n)).argsort(axis=1).argsort(axis=1)  # rank of row r in a random order
            ne = rng.integers(0, p + 1, G) if mixed else np.full(G, args.erasures)
            erased = ranks < ne[:, None]  # ne[g] distinct rows, uniform
            masks = np.zeros(G, np.uint64)
            for r in range(n):
                masks |= (~erased[:, r]).astype(np.uint64) << np.uint64(r)
            gi, ri = np.nonzero(erased)
            buf[gi, ri] = 0
            times = []
            for k in range(4):
                t0 = time.perf_counter()
                rc = enc.reconstruct_host(buf, masks, S)
                times.append(time.perf_counter() - t0)
                assert rc == 0, rc
            t_rec = sorted(times[1:])[1]
            ok = bool(torch.equal(torch.from_numpy(buf).to(dev)[:, :, :S], ref[:, :, :S]))
            del ref
            e_tot = int(ne.sum())
            lossy = int((ne > 0).sum())
            b_enc = G * n * S
            b_rec = lossy * d * S + e_tot * S
            key = f"{d}+{p}x{S}"
            res[key] = {
                "groups": G, "erasures": "U[0,%d] per group" % p if mixed else f"{args.erasures} per group",
                "encode_ms": round(t_enc * 1e3, 3), "encode_GBps": round(b_enc / t_enc / 1e9, 2),
                "encode_pcie_GBps": round(G * (d * pitch + p * S) / t_enc / 1e9, 2),
                "reconstruct_ms": round(t_rec * 1e3, 3), "reconstruct_GBps": round(b_rec / t_rec / 1e9, 2),
                "reconstruct_pcie_GBps": round(b_rec / t_rec / 1e9, 2),
                "verify_round_trip": ok}
        finally:
            fec.host_free(raw)
            enc.close()
    res["note"] = ("pinned host batches, group-major; GBps = algorithmic bytes ((d+p)*S encode, (d+e)*S per lossy "
                   "group reconstruct) / wall time of the synchronous call; pcie_GBps = bytes crossing PCIe (encode: "
                   "d padded rows in + p rows out, staged; reconstruct: d survivor rows in + e rows out, zero-copy)")
    return res


def per_call_leg(args, dev_index):
    """The drop-in route's latency (north_star: unchanged Encode / Reconstruct
    signatures, ugo/fec.go:202,238): one (10+3) group per call, as the cgo shim
    of INTEGRATION.md §2 makes it -- a pinned stage at the 16-B pitch, groups =
    1 -- with the 1470-B calcECC window for Encode and ugo's 1476-B buffers and
    one lost data shard for Reconstruct.  Each call is made through the C-ABI
    (ctypes: ~1 us of Python call overhead included) 2,000 times after 200
    untimed, median per call; first on the launch path, then with the per-call
    service on (ugo_fec_service_start).  Verified: the service's parity and
    rebuilt shard equal the launch path's."""
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
    finally:
        fec.host_free(raw)
        enc.close()
    res["note"] = ("one (10+3) group per call through the C-ABI from Python (ctypes), the cgo shim's staging: "
                   "launch = one kernel launch + stream synchronize per call; service = ugo_fec_service_start "
                   "(a resident workgroup polls a pinned mailbox); one GFNI CPU core: ~0.67 us Encode, ~0.48 us "
                   "1-loss Reconstruct (DESIGN.md §4)")
    return res


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

    # 3. Secondary legs, after the main line's measurement (nothing in them
    #    feeds `value`): BASELINE configs[3] strong over the ranks, and at N = 1
    #    the PCIe-inclusive host path (configs[4] among it).
    batches = outs = shards = view = None
    torch.cuda.empty_cache()
    strong = strong_leg(args, enc, rank, world, dev, stream) if args.c4_total_groups > 0 else None
    host = host_path_leg(args, dev_index) if (world == 1 and not args.no_host_path) else None
    per_call = None
    if world == 1 and not args.no_host_path:
        try:  # a secondary leg: a failure here is reported in the line, never loses it
            per_call = per_call_leg(args, dev_index)
        except Exception as ex:  # noqa: BLE001
            per_call = {"error": repr(ex)[:300]}

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
                "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic,
                "note": f"achieved = algorithmic bytes per launch ({'(d+p)*S' if dom == 'encode' else '(d+e)*S'}"
                        f" per group x {G} groups) / avg kernel duration over a kernel-timing pass of the same "
                        f"{args.steps} steps right after the timed region, from hipExtLaunchKernel start/stop "
                        f"events on the launch stream (ms_per_step of that pass: "
                        f"{elapsed_timing_pass / args.steps * 1e3:.4f})"
                        + (f"; {traffic_note}" if traffic_note else "")}
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
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(args, d, p, S, n)
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
