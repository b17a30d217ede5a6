"""GPU parity at BASELINE configs[3]'s size and at the launch-slicing limits.

* configs[3] ("4M groups ... (10+3)x1350 B encode+decode"): the whole
  4,194,304-group batch on one MI355X, in the planar layout bench.py times.
  Its row stride is 4,194,304 x 1360 B = 5.7 GB, so every row past row 0 --
  and row 0 of every group past 3,158,064 -- sits past the 4 GiB offset: the
  64-bit addressing regime of the kernels (fec_kernels.hpp Batch strides,
  ugo_fec.cpp launch slicing).  Full-size round trip (the erased rows are
  zeroed in the batch first, so only a correct reconstruction can reproduce
  them), plus 512 groups -- including groups 0, G-1 and groups past 4 GiB --
  byte for byte against the oracle (encode and reconstruct).
* Launch slicing: a launch's work-item count is a uint32, and the wave-aligned
  kernels pad every group of a short-row code to a whole wave (1 chunk per
  row -> 64 lanes).  (40+8)x16 B at 2^26 + 4,096 groups (51.5 GB) is past the
  point where groups x 64 wraps 32 bits: every group must still be encoded
  and reconstructed (ugo_fec.cpp sized the slices from the
  unpadded count, and most groups' parity was silently never written).

Groups are independent codewords (/root/reference/ugo/fec.go:145-146), so a
batch of any size is the same computation per group; these tests pin that the
engine's slicing and 64-bit offsets keep it so.  Oracle = checker only.
"""
import numpy as np
import pytest
import torch

import rs_ref
from ugo_amd import fec

pytestmark = pytest.mark.gpu


def _sample_idx(G, k, seed, extra=()):
    rng = np.random.default_rng(seed)
    idx = set(int(x) for x in rng.choice(G, k, replace=False))
    idx |= {0, 1, G - 2, G - 1} | {int(x) for x in extra if 0 <= x < G}
    return np.array(sorted(idx), dtype=np.int64)


def test_configs3_4m_groups_round_trip_vs_oracle(gpu):
    """BASELINE configs[3] at N = 1: 4,194,304 groups of (10+3)x1350 in the
    planar [13][G][1360] layout (74.2 GB), encode then reconstruct_into with 2
    uniformly random erasures per group (bench.make_masks), as bench.py's
    strong_c4 leg times it."""
    import bench

    d, p, n, S, pitch, G = 10, 3, 13, 1350, 1360, 4194304
    enc = fec.New(d, p)
    gen = torch.Generator(device="cuda").manual_seed(0xC4)
    sh = torch.randint(0, 256, (n, G, pitch), dtype=torch.uint8, device="cuda", generator=gen)
    enc.encode_batch(sh, shard_size=S, shard_major=True)
    view = sh.transpose(0, 1)  # [G, n, pitch]
    past_4g = [4 * 2**30 // pitch + k for k in (0, 1, 777, 100000)]  # row 0 past the 4 GiB offset
    idx = _sample_idx(G, 512, 7, past_4g)
    ti = torch.as_tensor(idx, device="cuda")
    smp = view[ti].cpu().numpy()[:, :, :S].copy()  # encoded groups (before any erasure)
    want = smp.copy()
    want[:, d:] = 0
    rs_ref.c_encode(d, p, want)
    assert np.array_equal(smp, want), "encode differs from the oracle at 4M groups"

    masks, erased = bench.make_masks(G, n, 2, 0xC4 + 1000, "cuda")
    es = erased.sort(dim=1).values.cuda()
    gi = torch.arange(G, device="cuda")
    keep = [view[gi, es[:, j], :S].clone() for j in range(2)]  # the rows about to be erased
    for j in range(2):
        view[gi, es[:, j]] = 0  # only a correct reconstruction can bring them back
    out = torch.full((p, G, pitch), 0xA5, dtype=torch.uint8, device="cuda")
    st = torch.full((G,), -1, dtype=torch.int8, device="cuda")
    enc.reconstruct_into(sh, masks, out, shard_size=S, status=st, shard_major=True)
    torch.cuda.synchronize()
    assert bool((st == 0).all())
    for j in range(2):  # full-size round trip
        assert torch.equal(out[j, :, :S], keep[j]), f"output {j} differs from the erased rows"
    del keep
    assert bool((out[2] == 0xA5).all()), "slot past the erasures written"
    # oracle: reconstruct the sampled groups from the same erased input
    m = masks[ti].cpu().numpy().view(np.uint64)
    inp = view[ti].cpu().numpy()[:, :, :S].copy()
    rc, want_st = rs_ref.c_reconstruct(d, p, inp, m)
    assert rc == 0 and not want_st.any()
    o = out[:, ti, :S].cpu().numpy()
    er = es[ti].cpu().numpy()
    for k in range(len(idx)):
        for j in range(2):
            assert np.array_equal(o[j, k], inp[k, er[k, j]]), (idx[k], j)
            assert np.array_equal(o[j, k], want[k, er[k, j]]), (idx[k], j)


def test_short_row_wide_code_slicing_past_32_bits(gpu):
    """(40+8)x16 B at 2^26 + 4096 groups (planar, 51.5 GB): one row is a single
    16-B chunk, padded to a 64-lane wave per group by the wave-aligned kernel,
    so groups x 64 > 2^32.  Every group's parity is written (the last groups
    included) and every group reconstructs."""
    d, p, n, S = 40, 8, 48, 16
    G = 2**26 + 4096
    enc = fec.New(d, p)
    gen = torch.Generator(device="cuda").manual_seed(0x51)
    sh = torch.randint(0, 256, (n, G, S), dtype=torch.uint8, device="cuda", generator=gen)
    sentinel = 0x5A
    sh[d:] = sentinel
    enc.encode_batch(sh, shard_size=S, shard_major=True)
    torch.cuda.synchronize()
    view = sh.transpose(0, 1)
    # no group keeps the sentinel parity (a 16-B row of 0x5A by chance: ~2^-128)
    untouched = (sh[d:] == sentinel).all(dim=2).all(dim=0)
    assert not bool(untouched.any()), f"{int(untouched.sum())} groups never encoded"
    idx = _sample_idx(G, 512, 11, [2**25 - 1, 2**25, 2**26 - 1, 2**26, G - 4096])
    ti = torch.as_tensor(idx, device="cuda")
    smp = view[ti].cpu().numpy().copy()
    want = smp.copy()
    want[:, d:] = 0
    rs_ref.c_encode(d, p, want)
    assert np.array_equal(smp, want), "encode differs from the oracle"
    # 2 erasures per group, a data row and a parity row, pattern varying with g
    r0 = (gi := torch.arange(G, device="cuda")) % d
    r1 = d + (gi * 7 + 3) % p
    full = (1 << n) - 1
    masks = (torch.full((G,), full, dtype=torch.int64, device="cuda")
             ^ (torch.ones_like(gi) << r0) ^ (torch.ones_like(gi) << r1))
    keep = [view[gi, r0].clone(), view[gi, r1].clone()]
    view[gi, r0] = 0
    view[gi, r1] = 0
    out = torch.full((p, G, S), 0xA5, dtype=torch.uint8, device="cuda")
    st = torch.full((G,), -1, dtype=torch.int8, device="cuda")
    enc.reconstruct_into(sh, masks, out, shard_size=S, status=st, shard_major=True)
    torch.cuda.synchronize()
    assert bool((st == 0).all())
    assert torch.equal(out[0], keep[0]) and torch.equal(out[1], keep[1]), "round trip failed"
    m = masks[ti].cpu().numpy().view(np.uint64)
    inp = view[ti].cpu().numpy().copy()
    rc, want_st = rs_ref.c_reconstruct(d, p, inp, m)
    assert rc == 0 and not want_st.any()
    o = out[:, ti].cpu().numpy()
    r0h, r1h = r0[ti].cpu().numpy(), r1[ti].cpu().numpy()
    for k in range(len(idx)):
        assert np.array_equal(o[0, k], inp[k, r0h[k]]) and np.array_equal(o[1, k], inp[k, r1h[k]]), idx[k]
