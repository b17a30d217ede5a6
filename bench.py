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
the state a fresh batch of packets arrives in.  Algorithmic bytes per group: encode (d+p)*S,
reconstruct (d+e)*S; value = sum over ranks / max-over-ranks time, in GiB/s.

Multi-GPU (torchrun, one process per GPU): packet groups are independent, so
each rank owns its own batch (weak scaling) -- or a contiguous 1/N slice of
--total-groups (strong scaling) -- and no data-path collective runs; only the
timing barrier and a max-reduction.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--groups G]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from ugo_amd import fec  # noqa: E402
from ugo_amd.shard import dist_env, partition  # noqa: E402

METRIC = "FEC encode+decode GiB/s device-resident, (10+3)×1350B groups; %HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak, GB/s (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=50,
                    help="untimed steps; the clocks take ~20 ms of load to reach steady state")
    ap.add_argument("--groups", type=int, default=65536, help="groups per GPU (weak scaling)")
    ap.add_argument("--total-groups", type=int, default=0, help="if set: strong scaling over this many groups")
    ap.add_argument("--data-shards", type=int, default=10)
    ap.add_argument("--parity-shards", type=int, default=3)
    ap.add_argument("--shard-size", type=int, default=1350)
    ap.add_argument("--pitch", type=int, default=0, help="row pitch in HBM (default: shard size rounded to 16)")
    ap.add_argument("--erasures", type=int, default=2)
    ap.add_argument("--batches", type=int, default=2,
                    help="rotate the steps over this many independent batches per GPU (step k works on batch "
                         "k mod B). With B >= 2 every step meets a cold batch, as a fresh batch of packets is: "
                         "none of its lines are in the 256-MB Infinity Cache. B = 1 re-runs one batch, and the "
                         "cache then absorbs part of the rewritten parity (DESIGN.md §4)")
    ap.add_argument("--layout", choices=["planar", "interleaved"], default="planar",
                    help="planar = shard-major [d+p][G][pitch] batch; interleaved = [G][d+p][pitch]")
    ap.add_argument("--decode", choices=["inplace", "into"], default="into",
                    help="inplace = ugo_fec_reconstruct_strided (erased rows rebuilt inside the batch); into = "
                         "ugo_fec_reconstruct_into (erased rows written to a separate [p][G][pitch] output batch, "
                         "the fresh buffers klauspost's Reconstruct gives ugo's nil shards)")
    ap.add_argument("--seed", type=int, default=0x5EED)
    ap.add_argument("--cpu-baseline-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-threads", type=int, default=16,
                    help="CPU baseline threads (the GPU box's CPU share is 16; capped at os.cpu_count())")
    ap.add_argument("--cpu-simd", type=int, default=-1,
                    help="CPU baseline SIMD level: -1 best available, 0 scalar, 1 AVX2, 2 AVX-512 GFNI")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"),
                    help="per-launch HBM bytes from rocprofv3 PMC passes (tools/pmc_traffic.py)")
    return ap.parse_args()


def make_masks(G, n, e, seed, device):
    """Presence masks with exactly e distinct erased shards per group."""
    gen = torch.Generator(device="cpu").manual_seed(seed)
    keys = torch.rand((G, n), generator=gen)
    erased = keys.argsort(dim=1)[:, :e]  # e distinct indices, uniform over C(n, e)
    masks = torch.full((G,), (1 << n) - 1, dtype=torch.int64)
    for j in range(e):
        masks ^= (1 << erased[:, j]).to(torch.int64)
    return masks.to(device), erased


def cpu_baseline(args, d, p, S, n, sample_groups=4096):
    """The CPU oracle (oracle/rs_oracle.c: the upstream algorithm, with the
    upstream library's SIMD strategy -- AVX-512 GFNI affine or AVX2 nibble
    tables, fused multi-output column blocks, per-pattern inverse cache) timed
    on this host's cores on a bounded sample of the same workload."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import rs_ref  # checker / CPU baseline only

    rs_ref.load_c_oracle()
    level = rs_ref.set_simd(args.cpu_simd)
    threads = max(1, min(args.cpu_threads, os.cpu_count() or 1))
    rng = np.random.default_rng(args.seed)
    sh = rng.integers(0, 256, size=(sample_groups, n, S), dtype=np.uint8)
    masks = np.full(sample_groups, (1 << n) - 1, np.uint64)
    for g in range(sample_groups):
        for r in rng.choice(n, args.erasures, replace=False):
            masks[g] &= ~np.uint64(1 << int(r))
    t0 = time.perf_counter()
    passes = 0
    try:
        while True:
            rs_ref.c_encode(d, p, sh, threads=threads)
            rs_ref.c_reconstruct(d, p, sh, masks, threads=threads)
            passes += 1
            el = time.perf_counter() - t0
            if el >= args.cpu_baseline_seconds:
                break
    finally:
        rs_ref.set_simd(0)
    per_pass = sample_groups * ((d + p) * S + (d + args.erasures) * S)
    return {"value": round(per_pass * passes / el / 2**30, 4), "unit": "GiB/s", "cores": threads,
            "kind": "port",
            "sample": f"{sample_groups} groups ({d}+{p})x{S}B, encode + {args.erasures}-erasure reconstruct, "
                      f"{passes} passes in {el:.1f}s on {threads} threads, oracle/rs_oracle.c "
                      f"[{rs_ref.SIMD_NAMES[level]}] (C restatement of the klauspost algorithm and its SIMD "
                      f"strategy; the Go reference cannot run: no Go toolchain)"}


def main():
    args = parse()
    rank, local_rank, world = dist_env()
    if world > 1:
        dist.init_process_group("nccl", init_method="env://")
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    d, p, S = args.data_shards, args.parity_shards, args.shard_size
    n = d + p
    pitch = args.pitch or (S + 15) // 16 * 16
    if args.total_groups:
        g0, g1 = partition(args.total_groups, world, rank)
        G = g1 - g0
        scaling = "strong"
    else:
        G = args.groups
        g0 = rank * G
        scaling = "weak"
    e = args.erasures

    enc = fec.New(d, p, device=local_rank)
    gen = torch.Generator(device=dev).manual_seed(args.seed + rank)
    planar = args.layout == "planar"
    shape = (n, G, pitch) if planar else (G, n, pitch)
    nb = max(1, args.batches)
    batches = [torch.randint(0, 256, shape, dtype=torch.uint8, device=dev, generator=gen) for _ in range(nb)]
    shards = batches[0]
    masks, erased = make_masks(G, n, e, args.seed + 1000 + rank, dev)
    into = args.decode == "into"
    # one output batch per input batch, so every step's outputs are cold too
    outs = [torch.zeros((p, G, pitch), dtype=torch.uint8, device=dev) for _ in range(nb)] if into else None
    stream = torch.cuda.current_stream()
    cur = [0]

    def step():
        i = cur[0] % nb
        b = batches[i]
        cur[0] += 1
        enc.encode_batch(b, shard_size=S, stream=stream, shard_major=planar)
        if into:
            enc.reconstruct_into(b, masks, outs[i], shard_size=S, stream=stream, shard_major=planar)
        else:
            enc.reconstruct_batch(b, masks, shard_size=S, stream=stream, shard_major=planar)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    # 1. The timed region (`value`): K steps of ordinary launches, barrier +
    #    synchronize on both sides, max over ranks.
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0

    # 2. Kernel-timing pass (`roofline`, `kernels`): the same K steps again with
    #    the library's launch timing on -- each launch issued with
    #    hipExtLaunchKernel start/stop events (ugo_fec_timing_begin), which carry
    #    the dispatch's own timestamps on the launch stream.  The events cost
    #    ~5 us per kernel boundary (tools/gap_probe.py: 374.8 vs 364.6 us per
    #    step), so the value pass above runs without them.
    enc.timing_begin(4 * args.steps + 16)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for k in range(args.steps):
        step()
    torch.cuda.synchronize()
    elapsed_timing_pass = time.perf_counter() - t1
    recs, untimed = enc.timing_end()
    kid = recs["kernel"]
    n_enc = int((kid == 1).sum())
    n_dec = int(np.isin(kid, (2, 3)).sum())
    assert n_enc >= args.steps and n_dec >= args.steps, (n_enc, n_dec)
    enc_ms = float(recs["ms"][kid == 1].sum()) / args.steps
    dec_ms = float(recs["ms"][np.isin(kid, (2, 3))].sum()) / args.steps  # apply (+ k_prepare for d+p > 16)

    t = torch.tensor([elapsed, enc_ms, dec_ms], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed, enc_ms_max, dec_ms_max = t.tolist()
    total_groups = G * world if scaling == "weak" else args.total_groups

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
            o = torch.full((p, G, pitch), 0xA5, dtype=torch.uint8, device=dev)
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
        okt = torch.tensor([int(ok_rt and ok_idem)], device=dev)
        if world > 1:
            dist.all_reduce(okt, op=dist.ReduceOp.MIN)
        verify["all_ranks_ok"] = bool(okt.item())

    if rank == 0:
        payload = G * d * S  # klauspost's convention: data bytes per call (BASELINE.md secondary column)
        kern = {
            "encode": {"avg_ms": round(enc_ms, 5), "bytes_per_launch": enc_bytes,
                       "GBps": round(enc_bytes / (enc_ms * 1e-3) / 1e9, 1),
                       "payload_GBps": round(payload / (enc_ms * 1e-3) / 1e9, 1),
                       "frac": round(enc_bytes / (enc_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)},
            "reconstruct": {"avg_ms": round(dec_ms, 5), "bytes_per_launch": dec_bytes,
                            "GBps": round(dec_bytes / (dec_ms * 1e-3) / 1e9, 1),
                            "payload_GBps": round(payload / (dec_ms * 1e-3) / 1e9, 1),
                            "frac": round(dec_bytes / (dec_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)},
        }
        dom = "encode" if enc_ms >= dec_ms else "reconstruct"
        traffic = None
        try:
            tj = json.load(open(args.traffic_json))
            key = f"{dom}:{d}+{p}x{S}/{pitch}:G{G}" + (":into" if into and dom == "reconstruct" else "")
            traffic = tj.get(key)
        except Exception:
            pass
        ach = kern[dom]["GBps"]
        roof = {"bound": "hbm", "kernel": dom, "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic,
                "note": f"achieved = algorithmic bytes per launch ({'(d+p)*S' if dom == 'encode' else '(d+e)*S'}"
                        f" per group x {G} groups) / avg kernel duration over a kernel-timing pass of the same "
                        f"{args.steps} steps right after the timed region, from hipExtLaunchKernel start/stop "
                        f"events on the launch stream (ms_per_step of that pass: "
                        f"{elapsed_timing_pass / args.steps * 1e3:.4f})"}
        out = {
            "metric": METRIC, "value": round(value, 3), "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
            "scaling": scaling, "vs_baseline": None, "dtype": "u8",
            "data": "synthetic: device-generated uniform random bytes (seeded), "
                    f"{e} distinct uniformly random erased shards per group",
            "config": {"workload": f"({d}+{p})x{S}B groups, encode + {e}-erasure reconstruct, device-resident, "
                                   f"{G} groups/GPU", "groups_per_gpu": G, "total_groups": total_groups,
                       "data_shards": d, "parity_shards": p, "shard_size": S, "pitch": pitch, "erasures": e,
                       "layout": "shard-major [d+p][G][pitch]" if planar else "group-major [G][d+p][pitch]",
                       "batches_per_gpu": nb, "decode": args.decode,
                       "parallelism": f"dp{world} (independent packet groups, no collective)"},
            "pct_hbm_roofline": round(step_bytes_all / world * args.steps / elapsed / (HBM_PEAK_GBS * 1e9), 4),
            "roofline": roof, "kernels": kern, "verify": verify,
        }
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(args, d, p, S, n)
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
