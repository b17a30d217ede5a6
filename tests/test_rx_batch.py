"""RX group assembly (SURVEY §8f rows 1 + 3): RC4 decrypt + FEC header decode +
group/slot placement on the GPU (ugo_fec_rx_assemble), then batch Reconstruct.

Checked against the oracle: packets produced by the restated ugo sender
(oracle/fec_ref.py), encrypted with the restated RC4 (oracle/rc4_ref.py,
pinned below by the classic published vectors), pushed through a lossy
channel; the expected batch is assembled on the CPU from the decrypted
packets and reconstructed with the C oracle.  Bit-exact comparison of the
whole planar batch, the presence masks, the per-group status and the stats.
"""
import os

import numpy as np
import pytest
import torch
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

import fec_ref
import rc4_ref
import rs_ref
from ugo_amd import fec

KEY = b"1234567890123456"  # ugo/listener.go:92, ugo/dial.go:132


def test_rc4_known_answers_and_product_keystream():
    assert rc4_ref.xor_stream(b"Key", b"Plaintext").hex() == "bbf316e8d940af0ad3"
    assert rc4_ref.xor_stream(b"Wiki", b"pedia").hex() == "1021bf0420"
    assert rc4_ref.xor_stream(b"Secret", b"Attack at dawn").hex() == "45a01f645fc35b383552544b9bf5"
    for key in (b"Key", b"Wiki", KEY):
        assert fec.rc4_keystream(key, 1536) == rc4_ref.keystream(key, 1536)


def _expected_placement(wire, G, n, S, pitch, first_group, frames=False):
    """The batch ugo's per-packet path builds from `wire` in ring order
    (decrypted packets): FEC.decode (ugo/fec.go:78-89), the flag filter of
    Conn.handlePacket (ugo/conn.go:395), the group/slot of input
    (ugo/fec.go:145,175), and its dedupe -- a seqid already queued drops the
    new packet, so the first copy stays (ugo/fec.go:123-129).  Returns the
    group-major batch, presence masks and stats [accepted, bad flag, out of
    window, too short, duplicate].  frames: a row holds the decrypted packet's
    first S + 6 bytes (ugo_fec_rx_assemble_frames: header, then the payload
    at column 6) instead of its payload."""
    want = np.zeros((G, n, pitch), np.uint8)
    masks = np.zeros(G, np.uint64)
    stats = [0, 0, 0, 0, 0]
    seen = set()
    for w in wire:
        if len(w) < 6:
            stats[3] += 1
            continue
        seq = int.from_bytes(w[:4], "little")
        flag = int.from_bytes(w[4:6], "little")
        if flag not in (0xF1, 0xF2):
            stats[1] += 1
            continue
        g = seq // n - first_group
        if not 0 <= g < G:
            stats[2] += 1
            continue
        if seq in seen:
            stats[4] += 1
            continue
        seen.add(seq)
        stats[0] += 1
        pl = w[:S + 6] if frames else w[6:6 + S]
        want[g, seq % n, :] = 0
        want[g, seq % n, :len(pl)] = np.frombuffer(pl, np.uint8)
        masks[g] |= np.uint64(1 << (seq % n))
    return want, masks, stats


def _ring(wire, slot):
    npk = len(wire)
    slots = np.zeros((npk, slot), np.uint8)
    lens = np.zeros(npk, np.uint16)
    for i, w in enumerate(wire):
        slots[i, :len(w)] = np.frombuffer(w, np.uint8)
        lens[i] = len(w)
    return slots, lens


def _packets(groups, seed, full_len):
    tx = fec_ref.FEC.new(128, 10, 3, clock=lambda: 0)
    rng = np.random.default_rng(seed)
    bufs = [bytearray(fec_ref.maxPacketSize) for _ in range(13)]
    out = []
    for _ in range(groups):
        maxsize = 0
        for k in range(10):
            L = 1476 if full_len else int(rng.integers(7, 1477))
            b = bytearray(rng.integers(0, 256, L, dtype=np.uint8).tobytes())
            tx.markData(b)
            bufs[k][:L] = b
            maxsize = max(maxsize, L)
            out.append(bytes(b))
        ecc = tx.calcECC(bufs, 6, maxsize)
        for k in range(3):
            tx.markFEC(ecc[k])
            out.append(bytes(ecc[k][:maxsize]))
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("full_len,encrypt,first_group,ring", [(True, True, 0, "device"), (False, True, 5, "device"),
                                                               (False, False, 0, "device"),
                                                               (False, True, 5, "pinned")])
def test_rx_assemble_and_reconstruct_vs_oracle(gpu, full_len, encrypt, first_group, ring):
    """ring = "pinned": the packet ring, lengths and pad stay in pinned host
    memory and the kernel reads them over PCIe (zero-copy)."""
    d, p, n, S, pitch, slot = 10, 3, 13, 1470, 1472, 1488
    total_groups, G = 300, 256
    pk = _packets(total_groups, 11, full_len)
    rng = np.random.default_rng(12)
    wire = []
    for w in pk:
        if rng.random() < 0.15:
            continue  # lost
        wire.append(w)
        if rng.random() < 0.05:
            wire.append(w)  # duplicate
        if rng.random() < 0.02:
            junk = bytearray(rng.integers(0, 256, 40, dtype=np.uint8).tobytes())
            junk[4:6] = b"\x00\x00"
            wire.append(bytes(junk))
    wire.append(b"\x01\x02")  # too short
    rng.shuffle(wire)
    ks = rc4_ref.keystream(KEY, slot)
    enc = [rc4_ref.xor_stream(KEY, w) if encrypt else w for w in wire]
    npk = len(enc)
    slots = np.zeros((npk, slot), np.uint8)
    lens = np.zeros(npk, np.uint16)
    for i, w in enumerate(enc):
        slots[i, :len(w)] = np.frombuffer(w, np.uint8)
        lens[i] = len(w)

    # expected: decode each (decrypted) packet on the CPU, place, reconstruct (oracle)
    want, masks, stats = _expected_placement(wire, G, n, S, pitch, first_group)
    exp = np.ascontiguousarray(want[:, :, :S])
    rc, exp_st = rs_ref.c_reconstruct(d, p, exp, masks, data_only=True)

    codec = fec.New(d, p)
    sh = torch.full((n, G, pitch), 0xAB, dtype=torch.uint8, device="cuda")  # garbage in unwritten rows
    present = torch.zeros(G, dtype=torch.int64, device="cuda")
    st = torch.zeros(5, dtype=torch.int32, device="cuda")
    if ring == "pinned":
        put = lambda t: t.pin_memory()  # noqa: E731
    else:
        put = lambda t: t.cuda()  # noqa: E731
    pad = put(torch.frombuffer(bytearray(ks), dtype=torch.uint8)) if encrypt else None
    codec.rx_assemble(put(torch.from_numpy(slots)), put(torch.from_numpy(lens.view(np.int16))), sh, present,
                      first_group=first_group, shard_size=S, pad=pad, stats=st)
    assert np.array_equal(present.cpu().numpy().view(np.uint64), masks)
    assert st.cpu().tolist() == stats
    raw = sh.cpu().numpy().transpose(1, 0, 2)
    for g in range(G):
        for r in range(n):
            if (int(masks[g]) >> r) & 1:
                assert not raw[g, r, S:].any(), (g, r)  # ABI 8: the last 16-B chunk written whole, zeros past S
            else:
                assert (raw[g, r] == 0xAB).all(), (g, r)  # rows no packet claimed stay untouched
    # the list form (ugo_fec_lossy_groups + ugo_fec_reconstruct_list): only the lossy groups, compact outputs
    lst, cnt = codec.lossy_groups(present, data_only=True)
    k = int(cnt.item())
    want_list = [g for g in range(G) if (~int(masks[g])) & ((1 << d) - 1)]
    assert lst.cpu().numpy()[:k].tolist() == want_list
    lout = torch.full((G, p, pitch), 0xA5, dtype=torch.uint8, device="cuda")
    lst_st = torch.full((G,), -1, dtype=torch.int8, device="cuda")
    codec.reconstruct_list(sh, present, lst, cnt, lout, shard_size=S, data_only=True, status=lst_st)
    lo, ls = lout.cpu().numpy(), lst_st.cpu().numpy()
    for j, g in enumerate(want_list):
        assert ls[j] == exp_st[g], (j, g)
        if exp_st[g] == 0:
            erased = [r for r in range(d) if not (int(masks[g]) >> r) & 1]
            for i, r in enumerate(erased):
                assert np.array_equal(lo[j, i, :S], exp[g, r]), (j, g, r)
    assert (lo[k:] == 0xA5).all()
    status = torch.full((G,), -1, dtype=torch.int8, device="cuda")
    codec.reconstruct_batch(sh, present, shard_size=S, data_only=True, status=status, shard_major=True)
    assert np.array_equal(status.cpu().numpy(), exp_st)
    got = sh.cpu().numpy().transpose(1, 0, 2)[:, :, :S]
    for g in range(G):
        m = int(masks[g])
        ok = bin(m).count("1") >= d
        for r in range(n):
            if (m >> r) & 1:
                assert np.array_equal(got[g, r], exp[g, r]), (g, r)       # placed packet
            elif r < d and ok:
                assert np.array_equal(got[g, r], exp[g, r]), (g, r)       # recovered data shard
    if full_len:  # consistent codewords: every recovered shard is the lost packet's payload
        nrec = 0
        for g in range(G):
            m = int(masks[g])
            if bin(m).count("1") < d:
                continue
            for r in range(d):
                if not (m >> r) & 1:
                    orig = pk[(g + first_group) * n + r][6:]
                    assert bytes(got[g, r]) == orig, (g, r)
                    nrec += 1
        assert nrec > 0


@pytest.mark.gpu
@pytest.mark.parametrize("full_len,encrypt,first_group,ring", [(True, True, 0, "device"), (False, True, 5, "device"),
                                                               (False, False, 0, "device"),
                                                               (False, True, 5, "pinned")])
def test_rx_assemble_frames_and_reconstruct_vs_oracle(gpu, full_len, encrypt, first_group, ring):
    """ugo_fec_rx_assemble_frames: each placed row is the decrypted packet
    (header in columns 0..5, payload from column 6, zeros to round_up(S + 6,
    16)); the lossy list, the list reconstruct and the in-place reconstruct run
    on the frame window (shard size S + 6), and the payload columns of every
    recovered row equal the oracle's Reconstruct (rs_ref) of the payload batch
    that fec_ref's decode + grouping builds -- the rows `input` appends to
    `recovered` (ugo/fec.go:190-207)."""
    d, p, n, S, slot = 10, 3, 13, 1470, 1488
    FS, pitch = S + 6, 1488
    total_groups, G = 300, 256
    pk = _packets(total_groups, 41, full_len)
    rng = np.random.default_rng(42 + first_group)
    wire = []
    for w in pk:
        if rng.random() < 0.15:
            continue  # lost
        wire.append(w)
        if rng.random() < 0.05:
            wire.append(w)  # duplicate
        if rng.random() < 0.02:
            junk = bytearray(rng.integers(0, 256, 40, dtype=np.uint8).tobytes())
            junk[4:6] = b"\x00\x00"
            wire.append(bytes(junk))
    wire.append(b"\x01\x02")  # too short
    rng.shuffle(wire)
    ks = rc4_ref.keystream(KEY, slot)
    slots, lens = _ring([rc4_ref.xor_stream(KEY, w) if encrypt else w for w in wire], slot)
    want_f, masks, stats = _expected_placement(wire, G, n, S, pitch, first_group, frames=True)
    want_p, masks_p, _ = _expected_placement(wire, G, n, S, (S + 15) // 16 * 16, first_group)
    assert np.array_equal(masks, masks_p)
    exp = np.ascontiguousarray(want_p[:, :, :S])
    _, exp_st = rs_ref.c_reconstruct(d, p, exp, masks, data_only=True)

    codec = fec.New(d, p)
    sh = torch.full((n, G, pitch), 0xAB, dtype=torch.uint8, device="cuda")
    present = torch.zeros(G, dtype=torch.int64, device="cuda")
    st = torch.zeros(5, dtype=torch.int32, device="cuda")
    put = (lambda t: t.pin_memory()) if ring == "pinned" else (lambda t: t.cuda())  # noqa: E731
    pad = put(torch.frombuffer(bytearray(ks), dtype=torch.uint8)) if encrypt else None
    codec.rx_assemble(put(torch.from_numpy(slots)), put(torch.from_numpy(lens.view(np.int16))), sh, present,
                      first_group=first_group, shard_size=S, pad=pad, stats=st, frames=True)
    assert np.array_equal(present.cpu().numpy().view(np.uint64), masks)
    assert st.cpu().tolist() == stats
    raw = sh.cpu().numpy().transpose(1, 0, 2)
    for g in range(G):
        for r in range(n):
            if (int(masks[g]) >> r) & 1:
                assert np.array_equal(raw[g, r], want_f[g, r]), (g, r)  # the frame, zeros to the row's end
            else:
                assert (raw[g, r] == 0xAB).all(), (g, r)
    lst, cnt = codec.lossy_groups(present, data_only=True)
    k = int(cnt.item())
    want_list = [g for g in range(G) if (~int(masks[g])) & ((1 << d) - 1)]
    assert lst.cpu().numpy()[:k].tolist() == want_list
    lout = torch.full((G, p, pitch), 0xA5, dtype=torch.uint8, device="cuda")
    lst_st = torch.full((G,), -1, dtype=torch.int8, device="cuda")
    codec.reconstruct_list(sh, present, lst, cnt, lout, shard_size=FS, data_only=True, status=lst_st)
    lo, ls = lout.cpu().numpy(), lst_st.cpu().numpy()
    nrec = 0
    for j, g in enumerate(want_list):
        assert ls[j] == exp_st[g], (j, g)
        if exp_st[g] == 0:
            erased = [r for r in range(d) if not (int(masks[g]) >> r) & 1]
            for i, r in enumerate(erased):
                assert np.array_equal(lo[j, i, 6:FS], exp[g, r]), (j, g, r)
                if full_len:  # consistent codewords: the lost packet's payload itself
                    assert bytes(lo[j, i, 6:FS]) == pk[(g + first_group) * n + r][6:], (j, g, r)
                nrec += 1
    assert nrec > 0
    status = torch.full((G,), -1, dtype=torch.int8, device="cuda")
    codec.reconstruct_batch(sh, present, shard_size=FS, data_only=True, status=status, shard_major=True)
    assert np.array_equal(status.cpu().numpy(), exp_st)
    got = sh.cpu().numpy().transpose(1, 0, 2)
    for g in range(G):
        m = int(masks[g])
        for r in range(n):
            if (m >> r) & 1:
                assert np.array_equal(got[g, r], want_f[g, r]), (g, r)  # present rows never written
            elif r < d and exp_st[g] == 0:
                assert np.array_equal(got[g, r, 6:FS], exp[g, r]), (g, r)


@pytest.mark.gpu
@pytest.mark.parametrize("encrypt,S,slot,frames", [(True, 1470, 1488, False), (False, 1470, 1488, False),
                                                   (True, 2000, 2016, False), (True, 3000, 3024, False),
                                                   (True, 1470, 1488, True), (True, 3000, 3024, True)])
def test_rx_assemble_first_copy_wins(gpu, encrypt, S, slot, frames):
    """Repeated seqids with DIFFERENT payloads and lengths (a replayed or
    corrupted packet with a valid header): the first copy in ring order is the
    one placed, as ugo's input keeps the queued packet and drops the new one
    (ugo/fec.go:123-129).  Copies sit next to each other (same wave), a wave
    apart and far apart; two runs in one process are identical.  S = 3000 runs
    the per-pass kernel (rows of more than 128 chunks); frames: the frame
    layout (k_rx_frame_h, and k_rx_frame_scatter at S = 3000)."""
    d, p, n = 10, 3, 13
    W = S + 6 if frames else S
    pitch = (W + 15) // 16 * 16
    G = 512
    rng = np.random.default_rng(77)
    maxlen = min(S + 6, slot)

    def pkt(seq, flag):
        L = int(rng.integers(6, maxlen + 1))
        b = bytearray(rng.integers(0, 256, L, dtype=np.uint8).tobytes())
        b[0:4] = seq.to_bytes(4, "little")
        b[4:6] = flag.to_bytes(2, "little")
        return bytes(b)

    wire = []
    for g in range(G):
        for r in range(n):
            if rng.random() < 0.1:
                continue
            seq = g * n + r
            flag = 0xF1 if r < d else 0xF2
            copies = 1 + int(rng.integers(0, 4)) if rng.random() < 0.3 else 1
            for _ in range(copies):
                wire.append(pkt(seq, flag))
    # ring order: mostly shuffled, with runs of adjacent copies kept together
    order = list(range(len(wire)))
    rng.shuffle(order)
    wire = [wire[i] for i in order]
    hot = pkt(5 * n + 2, 0xF1)
    wire[100:100] = [hot[:6] + bytes(rng.integers(0, 256, len(hot) - 6, dtype=np.uint8)) for _ in range(8)]
    wire.insert(0, pkt(7 * n + 12, 0xF2))
    wire.append(pkt(7 * n + 12, 0xF2))  # last copy of the first packet's seqid: dropped
    want, masks, stats = _expected_placement(wire, G, n, S, pitch, 0, frames)
    assert stats[4] > 50

    ks = rc4_ref.keystream(KEY, slot)
    enc = [rc4_ref.xor_stream(KEY, w) if encrypt else w for w in wire]
    slots, lens = _ring(enc, slot)
    codec = fec.New(d, p)
    pad = torch.frombuffer(bytearray(ks), dtype=torch.uint8).cuda() if encrypt else None
    ring = torch.from_numpy(slots).cuda()
    tl = torch.from_numpy(lens.view(np.int16)).cuda()
    runs = []
    for _ in range(2):
        sh = torch.full((n, G, pitch), 0xAB, dtype=torch.uint8, device="cuda")
        present = torch.zeros(G, dtype=torch.int64, device="cuda")
        st = torch.zeros(5, dtype=torch.int32, device="cuda")
        codec.rx_assemble(ring, tl, sh, present, shard_size=S, pad=pad, stats=st, frames=frames)
        runs.append((sh.cpu().numpy(), present.cpu().numpy().view(np.uint64), st.cpu().tolist()))
    for got, pres, st in runs:
        assert st == stats
        assert np.array_equal(pres, masks)
        g_major = got.transpose(1, 0, 2)
        for g in range(G):
            for r in range(n):
                if (int(masks[g]) >> r) & 1:
                    assert np.array_equal(g_major[g, r], want[g, r]), (g, r)
                else:
                    assert (g_major[g, r] == 0xAB).all(), (g, r)  # unclaimed rows untouched
    assert np.array_equal(runs[0][0], runs[1][0])


@pytest.mark.gpu
@pytest.mark.parametrize("encrypt,S,slot", [(True, 1470, 1488), (False, 3000, 3024)])
def test_rx_assemble_first_copy_wins_across_calls(gpu, encrypt, S, slot):
    """Several calls fill ONE batch (windows of one packet stream), with
    same-seqid, different-payload copies in later windows than the first: the
    batch keeps the first copy of the whole stream, as ugo's input keeps the
    queued packet (ugo/fec.go:123-129), and each call counts the later copies
    as duplicates.  The expected batch is the restated per-packet path run over
    the concatenated windows; the stats of a call are that path's counts over
    its own window, given what the earlier windows queued."""
    d, p, n = 10, 3, 13
    pitch = (S + 15) // 16 * 16
    G = 256
    rng = np.random.default_rng(91)
    maxlen = min(S + 6, slot)

    def pkt(seq, flag):
        L = int(rng.integers(6, maxlen + 1))
        b = bytearray(rng.integers(0, 256, L, dtype=np.uint8).tobytes())
        b[0:4] = seq.to_bytes(4, "little")
        b[4:6] = flag.to_bytes(2, "little")
        return bytes(b)

    stream = []
    for g in range(G):
        for r in range(n):
            if rng.random() < 0.15:
                continue
            seq = g * n + r
            copies = 1 + int(rng.integers(0, 3)) if rng.random() < 0.4 else 1
            stream += [pkt(seq, 0xF1 if r < d else 0xF2) for _ in range(copies)]
    order = rng.permutation(len(stream))
    stream = [stream[i] for i in order]
    cuts = [0, len(stream) // 5, len(stream) // 2, len(stream) * 4 // 5, len(stream)]
    windows = [stream[a:b] for a, b in zip(cuts, cuts[1:])]
    # a window whose packets ALL repeat seqids of earlier windows, with new payloads
    windows.append([pkt(int.from_bytes(w[:4], "little"), int.from_bytes(w[4:6], "little"))
                    for w in windows[0][:200]])
    want, masks, _ = _expected_placement(stream + windows[-1], G, n, S, pitch, 0)
    want_stats = []
    for k in range(len(windows)):
        prior = [w for win in windows[:k] for w in win]
        _, _, s_all = _expected_placement(prior + windows[k], G, n, S, pitch, 0)
        _, _, s_prior = _expected_placement(prior, G, n, S, pitch, 0)
        want_stats.append([a - b for a, b in zip(s_all, s_prior)])
    assert want_stats[-1][4] == 200 and want_stats[-1][0] == 0
    assert sum(s[4] for s in want_stats[1:4]) > 50  # cross-window copies in the middle windows too

    ks = rc4_ref.keystream(KEY, slot)
    pad = torch.frombuffer(bytearray(ks), dtype=torch.uint8).cuda() if encrypt else None
    codec = fec.New(d, p)
    sh = torch.full((n, G, pitch), 0xAB, dtype=torch.uint8, device="cuda")
    present = torch.zeros(G, dtype=torch.int64, device="cuda")
    for k, win in enumerate(windows):
        enc = [rc4_ref.xor_stream(KEY, w) if encrypt else w for w in win]
        slots, lens = _ring(enc, slot)
        st = torch.zeros(5, dtype=torch.int32, device="cuda")
        codec.rx_assemble(torch.from_numpy(slots).cuda(), torch.from_numpy(lens.view(np.int16)).cuda(), sh,
                          present, shard_size=S, pad=pad, stats=st)
        assert st.cpu().tolist() == want_stats[k], k
    assert np.array_equal(present.cpu().numpy().view(np.uint64), masks)
    got = sh.cpu().numpy().transpose(1, 0, 2)
    for g in range(G):
        for r in range(n):
            if (int(masks[g]) >> r) & 1:
                assert np.array_equal(got[g, r, :S], want[g, r, :S]), (g, r)
                assert not got[g, r, S:].any(), (g, r)  # ABI 8: whole 16-B chunks, zeros past S
            else:
                assert (got[g, r] == 0xAB).all(), (g, r)


@pytest.mark.gpu
@pytest.mark.parametrize("encrypt,first_group,max_out,pinned", [(True, 0, None, True), (True, 5, 40, True),
                                                                (False, 0, None, False)])
def test_rx_recover_host_vs_oracle(gpu, encrypt, first_group, max_out, pinned):
    """ugo_fec_rx_recover_host: a packet ring in host memory (loss, duplicates,
    junk, shuffled; >= 4 chunks) in, the recovered data shards out, row-compact
    in ugo's `recovered` order, against the oracle: placement (fec_ref decode +
    grouping), then Reconstruct (rs_ref) of each group with a lost data shard;
    stats and presence masks too.  max_out < the recovered count: only the
    first max_out shards come back, the count is still the total."""
    d, p, n, S, pitch, slot = 10, 3, 13, 1470, 1472, 1488
    total_groups, G = 300, 256
    pk = _packets(total_groups, 23, False)
    rng = np.random.default_rng(31 + first_group)
    wire = []
    for w in pk:
        if rng.random() < 0.12:
            continue  # lost
        wire.append(w)
        if rng.random() < 0.05:
            wire.append(w)  # duplicate
        if rng.random() < 0.02:
            junk = bytearray(rng.integers(0, 256, 40, dtype=np.uint8).tobytes())
            junk[4:6] = b"\x00\x00"
            wire.append(bytes(junk))
    rng.shuffle(wire)
    enc = [rc4_ref.xor_stream(KEY, w) if encrypt else w for w in wire]
    npk = len(enc)
    if pinned:
        slots = fec.host_alloc(npk * slot).reshape(npk, slot)
        lens = fec.host_alloc(npk * 2).view(np.uint16)
    else:
        slots, lens = np.zeros((npk, slot), np.uint8), np.zeros(npk, np.uint16)
    slots[:] = 0
    for i, w in enumerate(enc):
        slots[i, :len(w)] = np.frombuffer(w, np.uint8)
        lens[i] = len(w)
    want, masks, stats = _expected_placement(wire, G, n, S, pitch, first_group)
    exp = np.ascontiguousarray(want[:, :, :S])
    rc, exp_st = rs_ref.c_reconstruct(d, p, exp, masks, data_only=True)
    lossy = [g for g in range(G) if (~int(masks[g])) & ((1 << d) - 1)]
    # ugo's `recovered` (ugo/fec.go:203-207): every lost data shard of each group that Reconstruct
    # rebuilds, groups ascending, rows ascending; a group below d shards recovers nothing
    rec = [(g, r) for g in range(G) if exp_st[g] == 0 for r in range(d) if not (int(masks[g]) >> r) & 1]
    assert any(exp_st[g] != 0 for g in lossy), "the case should hold an unrecoverable lossy group"
    codec = fec.New(d, p)
    pres = np.zeros(G, np.uint64)
    nrec, index, out, got_stats = codec.rx_recover_host(
        slots, lens, S, G, first_group=first_group, pad=rc4_ref.keystream(KEY, slot) if encrypt else None,
        max_out=max_out, present_out=pres)
    assert nrec == len(rec)
    m = len(rec) if max_out is None else min(max_out, len(rec))
    assert index[:m].tolist() == [g * n + r for g, r in rec[:m]]
    assert np.array_equal(pres, masks)
    assert got_stats.tolist() == stats
    for j, (g, r) in enumerate(rec[:m]):
        assert np.array_equal(out[j, :S], exp[g, r]), (j, g, r)
    if pinned:
        fec.host_free(slots.reshape(-1))
        fec.host_free(lens.view(np.uint8))


@pytest.mark.gpu
def test_rx_recover_host_many_chunks_matches_device_path(gpu):
    """A ring past rx_recover_host's chunk cap (32 chunks per call; the chunks
    grow with the ring): 120,000 (10+3) groups, 5 % loss, shuffled, RC4 --
    ~1.48M packets, 2.2 GB pinned -- against the device-resident path
    (rx_assemble + lossy_groups + reconstruct_list, each checked against the
    oracle above): the recovered shards in `recovered` order, their places,
    the presence masks."""
    d, p, S, G, slot = 10, 3, 1470, 120000, 1488
    n, pitch = d + p, 1472
    gen = torch.Generator(device="cuda").manual_seed(5)
    seq = torch.arange(G * n, device="cuda", dtype=torch.int64)
    seq = seq[torch.rand(G * n, device="cuda", generator=gen) >= 0.05]
    seq = seq[torch.randperm(seq.numel(), device="cuda", generator=gen)]
    npk = seq.numel()
    assert npk > 32 * ((64 << 20) // slot)  # past the cap
    pad = fec.rc4_keystream(KEY, slot)
    dpad = torch.frombuffer(bytearray(pad), dtype=torch.uint8).cuda()
    w = torch.randint(0, 256, (npk, slot), dtype=torch.uint8, device="cuda", generator=gen)
    hdr = torch.zeros((npk, 6), dtype=torch.uint8, device="cuda")
    for b in range(4):
        hdr[:, b] = ((seq >> (8 * b)) & 0xFF).to(torch.uint8)
    hdr[:, 4] = torch.where(seq % n < d, 0xF1, 0xF2).to(torch.uint8)
    w[:, :6] = hdr ^ dpad[:6]
    lens = torch.full((npk,), 1476, dtype=torch.int16, device="cuda")
    codec = fec.New(d, p)
    bat = torch.empty((n, G, pitch), dtype=torch.uint8, device="cuda")
    pr = torch.zeros(G, dtype=torch.int64, device="cuda")
    codec.rx_assemble(w, lens, bat, pr, shard_size=S, pad=dpad)
    lst, cnt = codec.lossy_groups(pr, data_only=True)
    lo = torch.empty((G, p, pitch), dtype=torch.uint8, device="cuda")
    codec.reconstruct_list(bat, pr, lst, cnt, lo, shard_size=S, data_only=True)
    k = int(cnt.item())
    pm = pr[lst[:k].long()]
    lost = ((pm[:, None] >> torch.arange(d, device="cuda")) & 1) == 0
    have = ((pm[:, None] >> torch.arange(n, device="cuda")) & 1).sum(1)
    lost &= (have >= d)[:, None]
    jj, rr = torch.nonzero(lost, as_tuple=True)
    want_index = (lst[:k].long()[jj] * n + rr).cpu().numpy()
    want_rows = lo[:k][torch.arange(p, device="cuda")[None, :] < lost.sum(1)[:, None]]
    del bat, lo
    bufs = []
    try:
        ring = fec.host_alloc(npk * slot).reshape(npk, slot)
        bufs.append(ring)
        hl = fec.host_alloc(npk * 2).view(np.uint16)
        bufs.append(hl.view(np.uint8))
        torch.from_numpy(ring).copy_(w)
        hl[:] = 1476
        del w
        pres = np.zeros(G, np.uint64)
        nrec, index, out, stats = codec.rx_recover_host(ring, hl, S, G, pad=pad, present_out=pres)
        assert np.array_equal(pres.view(np.int64), pr.cpu().numpy())
        assert stats.tolist() == [npk, 0, 0, 0, 0]
        assert nrec == len(want_index)
        assert np.array_equal(index[:nrec].astype(np.int64), want_index)
        assert torch.equal(torch.from_numpy(out[:nrec, :S]).cuda(), want_rows[:, :S])
    finally:
        for a in bufs:
            fec.host_free(a)


@pytest.mark.gpu
def test_rx_assemble_rejects_pageable_host_memory(gpu):
    """A ring the GPU cannot reach is refused up front, not faulted on."""
    codec = fec.New(10, 3)
    ring = torch.zeros((64, 1488), dtype=torch.uint8)  # pageable
    lens = torch.full((64,), 1476, dtype=torch.int16, device="cuda")
    sh = torch.zeros((13, 8, 1472), dtype=torch.uint8, device="cuda")
    present = torch.zeros(8, dtype=torch.int64, device="cuda")
    with pytest.raises(fec.ErrInvalidArg):
        codec.rx_assemble(ring, lens, sh, present, shard_size=1470)


@pytest.mark.gpu
@settings(max_examples=int(os.environ.get("UGO_HYP_EXAMPLES_RX", "80")), deadline=None, derandomize=True,
          suppress_health_check=[HealthCheck.too_slow, HealthCheck.function_scoped_fixture])
@given(d=st.integers(1, 20), p=st.integers(1, 8), S=st.integers(1, 700), G=st.integers(1, 80),
       first_group=st.integers(0, 5), loss=st.floats(0, 0.5), dup=st.floats(0, 0.3), junk=st.floats(0, 0.1),
       encrypt=st.booleans(), seed=st.integers(0, 2**31 - 1), frames=st.booleans())
def test_rx_assemble_random_rings(gpu, d, p, S, G, first_group, loss, dup, junk, encrypt, seed, frames):
    """Random codes, shard sizes, windows and channels (loss, duplicates with
    different payloads, bad flags, short and out-of-window packets, any ring
    order): presence masks, stats and every placed row equal the per-packet
    reference path's (first copy of a seqid wins); rows no packet claimed stay
    untouched.  frames: the frame layout (ugo_fec_rx_assemble_frames), each row
    the packet's first S + 6 bytes, zeros to round_up(S + 6, 16)."""
    n = d + p
    W = S + 6 if frames else S  # bytes a placed row carries
    pitch = (W + 15) // 16 * 16
    slot = (S + 6 + 15) // 16 * 16
    rng = np.random.default_rng(seed)

    def pkt(seq, flag):
        L = int(rng.integers(6, S + 7))
        b = bytearray(rng.integers(0, 256, L, dtype=np.uint8).tobytes())
        b[0:4] = seq.to_bytes(4, "little")
        b[4:6] = flag.to_bytes(2, "little")
        return bytes(b)

    wire = []
    for g in range(first_group - 1, first_group + G + 1):  # one group either side of the window
        if g < 0:
            continue
        for r in range(n):
            if rng.random() < loss:
                continue
            for _ in range(1 + (int(rng.integers(1, 3)) if rng.random() < dup else 0)):
                wire.append(pkt(g * n + r, 0xF1 if r < d else 0xF2))
            if rng.random() < junk:
                wire.append(pkt(g * n + r, 0x77))  # bad flag
    if rng.random() < 0.5:
        wire.append(b"\x01\x02\x03")  # too short
    if not wire:
        return
    wire = [wire[i] for i in rng.permutation(len(wire))]
    want, masks, stats = _expected_placement(wire, G, n, S, pitch, first_group, frames)
    ks = rc4_ref.keystream(KEY, slot)
    enc = [rc4_ref.xor_stream(KEY, w) if encrypt else w for w in wire]
    slots, lens = _ring(enc, slot)
    codec = fec.New(d, p)
    sh = torch.full((n, G, pitch), 0xAB, dtype=torch.uint8, device="cuda")
    present = torch.zeros(G, dtype=torch.int64, device="cuda")
    stt = torch.zeros(5, dtype=torch.int32, device="cuda")
    pad = torch.frombuffer(bytearray(ks), dtype=torch.uint8).cuda() if encrypt else None
    codec.rx_assemble(torch.from_numpy(slots).cuda(), torch.from_numpy(lens.view(np.int16)).cuda(), sh, present,
                      first_group=first_group, shard_size=S, pad=pad, stats=stt, frames=frames)
    assert stt.cpu().tolist() == stats
    assert np.array_equal(present.cpu().numpy().view(np.uint64), masks)
    got = sh.cpu().numpy().transpose(1, 0, 2)
    for g in range(G):
        for r in range(n):
            if (int(masks[g]) >> r) & 1:
                assert np.array_equal(got[g, r, :W], want[g, r, :W]), (g, r)
                assert not got[g, r, W:].any(), (g, r)  # ABI 8: whole 16-B chunks, zeros past the row
            else:
                assert (got[g, r] == 0xAB).all(), (g, r)
