// asan_driver.cpp -- the C-ABI's host code under AddressSanitizer + UBSan
// ("ASan/UBSan on the C++ host path").  Built by
// tools/asan_build.sh together with every library source, host code
// instrumented, device code not (-Xarch_host -fsanitize=...), and run on the
// GPU box.  It drives every entry point family through its host logic --
// argument checks, staging, pinned zero-copy paths, the C++ FEC object in
// per-call and batched modes, RX/TX assembly -- and checks its own results
// by round trips (encode -> erase -> reconstruct == original; TX -> RX ==
// the sent payloads), so any memory error, UB or wrong byte stops it.
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "../include/ugo_fec.h"
#include "../include/ugo_fec_conn.h"

namespace {

int failures = 0;
#define EXPECT(c)                                                              \
  do {                                                                         \
    if (!(c)) {                                                                \
      std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c);        \
      ++failures;                                                              \
    }                                                                          \
  } while (0)

std::mt19937_64 rng(0x5EED);
uint8_t rb() { return static_cast<uint8_t>(rng()); }

void check_shards_cases() {
  size_t S = 0;
  const size_t a[3] = {10, 10, 10}, b[3] = {10, 0, 10}, c[3] = {0, 0, 0}, e[3] = {10, 9, 10};
  EXPECT(ugo_fec_check_shards(3, a, 0, &S) == UGO_FEC_OK && S == 10);
  EXPECT(ugo_fec_check_shards(3, b, 1, &S) == UGO_FEC_OK && S == 10);
  EXPECT(ugo_fec_check_shards(3, b, 0, &S) == UGO_FEC_ERR_SHARD_SIZE);
  EXPECT(ugo_fec_check_shards(3, c, 1, &S) == UGO_FEC_ERR_SHARD_NO_DATA);
  EXPECT(ugo_fec_check_shards(3, e, 1, &S) == UGO_FEC_ERR_SHARD_SIZE);
}

void null_args() {
  ugo_fec* ctx = nullptr;
  EXPECT(ugo_fec_create(0, 10, 3, nullptr) != UGO_FEC_OK);
  EXPECT(ugo_fec_create(0, 0, 3, &ctx) != UGO_FEC_OK && ctx == nullptr);
  EXPECT(ugo_fec_create(0, 200, 100, &ctx) != UGO_FEC_OK);
  EXPECT(ugo_fec_encode_host(nullptr, nullptr, 1, 10, 16) == UGO_FEC_ERR_INVALID_ARG);
  EXPECT(ugo_fec_reconstruct_host(nullptr, nullptr, nullptr, 1, 10, 16, 0, nullptr) == UGO_FEC_ERR_INVALID_ARG);
  ugo_fecconn* f = nullptr;
  EXPECT(ugo_fecconn_new(12, 10, 3, 0, &f) == UGO_FEC_ERR_INV_SHARD_NUM && f == nullptr);
  EXPECT(ugo_fecconn_input(nullptr, nullptr, 0, nullptr, nullptr, nullptr, 0, nullptr, nullptr) != UGO_FEC_OK);
  EXPECT(ugo_fec_strerror(UGO_FEC_ERR_SHARD_SIZE) != nullptr);
}

// encode -> erase up to p rows -> reconstruct == original, host buffers
void host_round_trip(int d, int p, size_t S, size_t G, bool pinned, bool svc = false) {
  const int n = d + p;
  const size_t pitch = (S + 15) / 16 * 16 + (pinned ? 0 : 16);
  ugo_fec* ctx = nullptr;
  EXPECT(ugo_fec_create(0, d, p, &ctx) == UGO_FEC_OK);
  if (!ctx) return;
  if (svc) EXPECT(ugo_fec_service_start(ctx, 300) == UGO_FEC_OK);  // the per-call service's host side
  const size_t bytes = G * n * pitch;
  uint8_t* buf = nullptr;
  std::vector<uint8_t> pageable;
  if (pinned) {
    void* v = nullptr;
    EXPECT(ugo_fec_host_alloc(bytes, &v) == UGO_FEC_OK);
    buf = static_cast<uint8_t*>(v);
  } else {
    pageable.resize(bytes);
    buf = pageable.data();
  }
  for (size_t i = 0; i < bytes; ++i) buf[i] = rb();
  EXPECT(ugo_fec_encode_host(ctx, buf, G, S, pitch) == UGO_FEC_OK);
  std::vector<uint8_t> ref(buf, buf + bytes);
  std::vector<uint64_t> mask(G);
  std::vector<int8_t> st(G, -1);
  for (size_t g = 0; g < G; ++g) {
    uint64_t m = (n >= 64 ? ~0ull : ((1ull << n) - 1));
    const int e = static_cast<int>(rng() % (p + 1));
    for (int k = 0; k < e; ++k) m &= ~(1ull << (rng() % n));
    mask[g] = m;
    for (int r = 0; r < n; ++r)
      if (!((m >> r) & 1)) std::memset(buf + (g * n + r) * pitch, 0xA5, S);
  }
  EXPECT(ugo_fec_reconstruct_host(ctx, buf, mask.data(), G, S, pitch, 0, st.data()) == UGO_FEC_OK);
  for (size_t g = 0; g < G; ++g) EXPECT(st[g] == 0);
  bool same = true;
  for (size_t g = 0; g < G && same; ++g)
    for (int r = 0; r < n && same; ++r)
      same = std::memcmp(buf + (g * n + r) * pitch, ref.data() + (g * n + r) * pitch, S) == 0;
  EXPECT(same);
  if (svc) EXPECT(ugo_fec_service_stop(ctx) == UGO_FEC_OK);
  if (pinned) ugo_fec_host_free(buf);
  ugo_fec_destroy(ctx);
}

// codes past 64 shards: ceil(n/64) presence words per group, host-built
// descriptors (round trip as above)
void host_round_trip_wide(int d, int p, size_t S, size_t G, bool pinned) {
  const int n = d + p;
  const size_t W = (n + 63) / 64, pitch = (S + 15) / 16 * 16;
  ugo_fec* ctx = nullptr;
  EXPECT(ugo_fec_create(0, d, p, &ctx) == UGO_FEC_OK);
  if (!ctx) return;
  const size_t bytes = G * n * pitch;
  uint8_t* buf = nullptr;
  std::vector<uint8_t> pageable;
  if (pinned) {
    void* v = nullptr;
    EXPECT(ugo_fec_host_alloc(bytes, &v) == UGO_FEC_OK);
    buf = static_cast<uint8_t*>(v);
  } else {
    pageable.resize(bytes);
    buf = pageable.data();
  }
  for (size_t i = 0; i < bytes; ++i) buf[i] = rb();
  EXPECT(ugo_fec_encode_host(ctx, buf, G, S, pitch) == UGO_FEC_OK);
  std::vector<uint8_t> ref(buf, buf + bytes);
  std::vector<uint64_t> mask(G * W, ~0ull);
  std::vector<int8_t> st(G, -1);
  for (size_t g = 0; g < G; ++g) {
    for (int r = n; r < static_cast<int>(64 * W); ++r) mask[g * W + r / 64] &= ~(1ull << (r % 64));
    const int e = static_cast<int>(rng() % (p + 1));
    for (int k = 0; k < e; ++k) {
      const int r = static_cast<int>(rng() % n);
      mask[g * W + r / 64] &= ~(1ull << (r % 64));
      std::memset(buf + (g * n + r) * pitch, 0xA5, S);
    }
  }
  EXPECT(ugo_fec_reconstruct_host(ctx, buf, mask.data(), G, S, pitch, 0, st.data()) == UGO_FEC_OK);
  for (size_t g = 0; g < G; ++g) EXPECT(st[g] == 0);
  EXPECT(std::memcmp(buf, ref.data(), bytes) == 0);
  if (pinned) ugo_fec_host_free(buf);
  ugo_fec_destroy(ctx);
}

// the FEC object: TX by markData / calcECC / markFEC over reused buffers, RX
// over a lossy, duplicating channel per call and batched -- same recovered
// sequence, and every lost full-length payload comes back
void fec_object(int batch, unsigned flags = 0, bool svc = false) {
  const int d = 10, p = 3, n = 13;
  const size_t L = UGO_FEC_MAX_PACKET;
  ugo_fecconn *tx = nullptr, *rx1 = nullptr, *rx2 = nullptr;
  EXPECT(ugo_fecconn_new(128, d, p, 0, &tx) == UGO_FEC_OK);
  EXPECT(ugo_fecconn_new(128, d, p, 0, &rx1) == UGO_FEC_OK);
  EXPECT(ugo_fecconn_new(128, d, p, 0, &rx2) == UGO_FEC_OK);
  if (!tx || !rx1 || !rx2) return;
  if (svc) {  // calcECC and rx1's per-call recovery through the per-call service
    EXPECT(ugo_fecconn_service(tx, 0) == UGO_FEC_OK);
    EXPECT(ugo_fecconn_service(rx1, 300) == UGO_FEC_OK);
  }
  std::vector<uint8_t> out1(size_t(batch + 1) * d * L), out2(size_t(2 * batch + 1) * d * L);
  int nrec = 0;
  size_t rl = 0;
  EXPECT(ugo_fecconn_set_batch_ex(rx2, batch, flags, out2.data(), out2.size(), &nrec, &rl) == UGO_FEC_OK);
  std::vector<std::vector<uint8_t>> grp(n, std::vector<uint8_t>(L));
  std::vector<std::vector<uint8_t>> wire, sent;
  for (int g = 0; g < 40; ++g) {
    for (int k = 0; k < d; ++k) {
      for (auto& x : grp[k]) x = rb();
      EXPECT(ugo_fecconn_mark_data(tx, grp[k].data()) == UGO_FEC_OK);
      sent.push_back(grp[k]);
    }
    std::vector<uint8_t*> ptrs(n);
    std::vector<size_t> lens(n, L);
    for (int k = 0; k < n; ++k) ptrs[k] = grp[k].data();
    EXPECT(ugo_fecconn_calc_ecc(tx, ptrs.data(), lens.data(), n, 6, static_cast<int>(L)) == UGO_FEC_OK);
    for (int k = d; k < n; ++k) EXPECT(ugo_fecconn_mark_fec(tx, grp[k].data()) == UGO_FEC_OK);
    for (int k = 0; k < n; ++k) {
      if (rng() % 100 < 12) continue;  // lost
      wire.push_back(grp[k]);
      if (rng() % 100 < 5) wire.push_back(grp[k]);  // duplicated
    }
  }
  std::vector<std::vector<uint8_t>> rec1, rec2;
  for (const auto& w : wire) {
    uint32_t seq;
    uint16_t flag;
    EXPECT(ugo_fecconn_input(rx1, w.data(), w.size(), &seq, &flag, out1.data(), out1.size(), &nrec, &rl) ==
           UGO_FEC_OK);
    for (int i = 0; i < nrec; ++i) rec1.emplace_back(out1.data() + i * L, out1.data() + i * L + rl);
    EXPECT(ugo_fecconn_input(rx2, w.data(), w.size(), &seq, &flag, out2.data(), out2.size(), &nrec, &rl) ==
           UGO_FEC_OK);
    for (int i = 0; i < nrec; ++i) rec2.emplace_back(out2.data() + i * L, out2.data() + i * L + rl);
  }
  EXPECT(ugo_fecconn_flush(rx2, out2.data(), out2.size(), &nrec, &rl) == UGO_FEC_OK);
  for (int i = 0; i < nrec; ++i) rec2.emplace_back(out2.data() + i * L, out2.data() + i * L + rl);
  size_t a = 0, b = 0;
  EXPECT(ugo_fecconn_rx_len(rx1, &a) == UGO_FEC_OK && ugo_fecconn_rx_len(rx2, &b) == UGO_FEC_OK && a == b);
  EXPECT(rec1 == rec2);
  EXPECT(!rec1.empty());
  for (const auto& r : rec1) {  // a recovered shard is a sent payload (packet bytes [6, L))
    bool found = false;
    for (const auto& s : sent)
      if (std::memcmp(s.data() + 6, r.data(), L - 6) == 0) {
        found = true;
        break;
      }
    EXPECT(found);
  }
  ugo_fecconn_free(tx);
  ugo_fecconn_free(rx1);
  ugo_fecconn_free(rx2);
}

// TX assembly -> RX assembly -> data-only reconstruct into: the data packets'
// payloads come back, pinned buffers used zero-copy
void tx_rx_batch() {
  const int d = 10, p = 3, n = 13;
  const size_t G = 64, max_len = 1476, slot = 1488, S = max_len - 6, pitch = 1472;
  ugo_fec* ctx = nullptr;
  EXPECT(ugo_fec_create(0, d, p, &ctx) == UGO_FEC_OK);
  if (!ctx) return;
  auto pin = [](size_t bytes) {
    void* v = nullptr;
    EXPECT(ugo_fec_host_alloc(bytes, &v) == UGO_FEC_OK);
    return static_cast<uint8_t*>(v);
  };
  uint8_t* pkts = pin(G * d * slot);
  uint8_t* wire = pin(G * n * slot);
  auto* lens = reinterpret_cast<uint16_t*>(pin(G * d * 2));
  auto* wlens = reinterpret_cast<uint16_t*>(pin(G * n * 2));
  auto* status = reinterpret_cast<int8_t*>(pin(G));
  uint8_t* pad = pin(slot);
  EXPECT(ugo_fec_rc4_keystream(reinterpret_cast<const uint8_t*>("1234567890123456"), 16, pad, slot) == UGO_FEC_OK);
  for (size_t i = 0; i < G * d * slot; ++i) pkts[i] = rb();
  for (size_t i = 0; i < G * d; ++i) lens[i] = static_cast<uint16_t>(max_len);
  EXPECT(ugo_fec_tx_assemble(ctx, pkts, slot, lens, G, 0, pad, max_len, wire, slot, wlens, status, nullptr) ==
         UGO_FEC_OK);
  EXPECT(hipDeviceSynchronize() == hipSuccess);
  for (size_t g = 0; g < G; ++g) EXPECT(status[g] == 0);
  // drop one data packet per group from the ring
  std::vector<size_t> keep;
  for (size_t g = 0; g < G; ++g)
    for (int r = 0; r < n; ++r)
      if (r != static_cast<int>(g % d)) keep.push_back(g * n + r);
  uint8_t* ring = pin(keep.size() * slot);
  auto* rlens = reinterpret_cast<uint16_t*>(pin(keep.size() * 2));
  for (size_t i = 0; i < keep.size(); ++i) {
    std::memcpy(ring + i * slot, wire + keep[i] * slot, slot);
    rlens[i] = wlens[keep[i]];
  }
  uint8_t* shards = pin(n * G * pitch);
  auto* present = reinterpret_cast<uint64_t*>(pin(G * 8));
  auto* stats = reinterpret_cast<uint32_t*>(pin(5 * 4));
  std::memset(present, 0, G * 8);
  std::memset(stats, 0, 20);
  EXPECT(ugo_fec_rx_assemble(ctx, ring, slot, rlens, keep.size(), pad, 0, G, shards, S, G * pitch, pitch, present,
                             stats, nullptr) == UGO_FEC_OK);
  EXPECT(hipDeviceSynchronize() == hipSuccess);
  EXPECT(stats[0] == keep.size());
  uint8_t* out = pin(p * G * pitch);
  EXPECT(ugo_fec_reconstruct_into(ctx, shards, present, G, S, G * pitch, pitch, out, G * pitch, pitch,
                                  UGO_FEC_RECONSTRUCT_DATA_ONLY, status, nullptr) == UGO_FEC_OK);
  EXPECT(hipDeviceSynchronize() == hipSuccess);
  bool same = true;
  for (size_t g = 0; g < G && same; ++g) {
    const size_t k = g % d;  // the lost data packet: output 0 of its group
    same = std::memcmp(out + g * pitch, pkts + (g * d + k) * slot + 6, S) == 0;
  }
  EXPECT(same);
  // the same recovery from a row-pointer table over the assembled batch (pinned, read in place)
  auto* rows = reinterpret_cast<uint64_t*>(pin(G * n * 8));
  uint8_t* out2 = pin(p * G * pitch);
  for (size_t g = 0; g < G; ++g)
    for (int r = 0; r < n; ++r) {
      void* dv = nullptr;
      EXPECT(ugo_fec_device_address(ctx, shards + r * G * pitch + g * pitch, &dv) == UGO_FEC_OK);
      rows[g * n + r] = reinterpret_cast<uint64_t>(dv);
    }
  EXPECT(ugo_fec_reconstruct_rows(ctx, reinterpret_cast<const uint8_t* const*>(rows), present, G, S, out2, G * pitch,
                                  pitch, UGO_FEC_RECONSTRUCT_DATA_ONLY, status, nullptr) == UGO_FEC_OK);
  EXPECT(hipDeviceSynchronize() == hipSuccess);
  for (size_t g = 0; g < G; ++g) EXPECT(status[g] == 0 && std::memcmp(out2 + g * pitch, out + g * pitch, S) == 0);
  ugo_fec_host_free(rows);
  ugo_fec_host_free(out2);
  for (uint8_t* q : {pkts, wire, reinterpret_cast<uint8_t*>(lens), reinterpret_cast<uint8_t*>(wlens),
                     reinterpret_cast<uint8_t*>(status), pad, ring, reinterpret_cast<uint8_t*>(rlens), shards,
                     reinterpret_cast<uint8_t*>(present), reinterpret_cast<uint8_t*>(stats), out})
    ugo_fec_host_free(q);
  ugo_fec_destroy(ctx);
}

// round 5: the lossy-group list + list reconstruct on a device batch, and
// the host-memory RX / TX paths (pinned and pageable buffers, max_out below
// the count, the TX chunk cap): results against tx_assemble / the data they
// were built from
void host_rx_tx_paths(bool pinned) {
  const int d = 10, p = 3, n = 13;
  const size_t G = 200, max_len = 1476, slot = 1488, S = max_len - 6, pitch = 1472;
  ugo_fec* ctx = nullptr;
  EXPECT(ugo_fec_create(0, d, p, &ctx) == UGO_FEC_OK);
  if (!ctx) return;
  std::vector<void*> owned;
  auto buf = [&](size_t bytes) {
    void* v = nullptr;
    if (pinned) {
      EXPECT(ugo_fec_host_alloc(bytes, &v) == UGO_FEC_OK);
    } else {
      v = std::calloc(bytes, 1);
    }
    owned.push_back(v);
    return static_cast<uint8_t*>(v);
  };
  uint8_t* pkts = buf(G * d * slot);
  auto* lens = reinterpret_cast<uint16_t*>(buf(G * d * 2));
  uint8_t* wire = buf(G * n * slot);
  auto* wlens = reinterpret_cast<uint16_t*>(buf(G * n * 2));
  auto* status = reinterpret_cast<int8_t*>(buf(G));
  uint8_t pad[1488];
  EXPECT(ugo_fec_rc4_keystream(reinterpret_cast<const uint8_t*>("1234567890123456"), 16, pad, slot) == UGO_FEC_OK);
  for (size_t i = 0; i < G * d * slot; ++i) pkts[i] = rb();
  for (size_t i = 0; i < G * d; ++i) lens[i] = static_cast<uint16_t>(i % 37 == 5 ? 700 : max_len);
  EXPECT(ugo_fec_tx_assemble_host(ctx, pkts, slot, lens, G, 0, pad, max_len, wire, slot, wlens, status) ==
         UGO_FEC_OK);
  for (size_t g = 0; g < G; ++g) EXPECT(status[g] == 0);
  // the other wire route (the kernel writes the pinned wire buffer through its mapping; a
  // pageable one falls back to the copy): the same packets and lengths
  EXPECT(ugo_fec_set_tx_host_route(ctx, 2) == UGO_FEC_ERR_INVALID_ARG);
  EXPECT(ugo_fec_set_tx_host_route(ctx, -1) == UGO_FEC_ERR_INVALID_ARG);
  EXPECT(ugo_fec_set_tx_host_route(ctx, 1) == UGO_FEC_OK);
  {
    uint8_t* wire2 = buf(G * n * slot);
    auto* wlens2 = reinterpret_cast<uint16_t*>(buf(G * n * 2));
    EXPECT(ugo_fec_tx_assemble_host(ctx, pkts, slot, lens, G, 0, pad, max_len, wire2, slot, wlens2, nullptr) ==
           UGO_FEC_OK);
    for (size_t i = 0; i < G * n; ++i) {
      EXPECT(wlens2[i] == wlens[i]);
      EXPECT(std::memcmp(wire2 + i * slot, wire + i * slot, wlens[i]) == 0);
    }
  }
  EXPECT(ugo_fec_set_tx_host_route(ctx, 0) == UGO_FEC_OK);
  // the low-priority copy stream, switched on between calls (the stream is replaced): same packets
  EXPECT(ugo_fec_set_host_copy_queue(ctx, 2) == UGO_FEC_ERR_INVALID_ARG);
  EXPECT(ugo_fec_set_host_copy_queue(ctx, 1) == UGO_FEC_OK);
  {
    uint8_t* wire3 = buf(G * n * slot);
    auto* wlens3 = reinterpret_cast<uint16_t*>(buf(G * n * 2));
    EXPECT(ugo_fec_tx_assemble_host(ctx, pkts, slot, lens, G, 0, pad, max_len, wire3, slot, wlens3, nullptr) ==
           UGO_FEC_OK);
    for (size_t i = 0; i < G * n; ++i) {
      EXPECT(wlens3[i] == wlens[i]);
      EXPECT(std::memcmp(wire3 + i * slot, wire + i * slot, wlens[i]) == 0);
    }
  }
  // the ring: every group loses data packet g % d, group 7 loses 4 packets (below d shards)
  std::vector<size_t> keep;
  for (size_t g = 0; g < G; ++g)
    for (int r = 0; r < n; ++r)
      if (r != static_cast<int>(g % d) && !(g == 7 && r < 4)) keep.push_back(g * n + r);
  uint8_t* ring = buf(keep.size() * slot);
  auto* rlens = reinterpret_cast<uint16_t*>(buf(keep.size() * 2));
  for (size_t i = 0; i < keep.size(); ++i) {
    std::memcpy(ring + i * slot, wire + keep[i] * slot, slot);
    rlens[i] = wlens[keep[i]];
  }
  for (size_t max_out : {size_t(3 * G), size_t(17), size_t(0)}) {
    uint8_t* out = buf(3 * G * pitch);
    auto* index = reinterpret_cast<uint32_t*>(buf(3 * G * 4));
    auto* present = reinterpret_cast<uint64_t*>(buf(G * 8));
    uint32_t stats[5] = {};
    size_t nrec = 0;
    EXPECT(ugo_fec_rx_recover_host(ctx, ring, slot, rlens, keep.size(), pad, 0, G, S, present, stats, out, pitch,
                                   max_out, index, &nrec) == UGO_FEC_OK);
    EXPECT(nrec == G - 1);  // group 7 recovers nothing
    EXPECT(stats[0] == keep.size());
    const size_t m = std::min(nrec, max_out);
    for (size_t r = 0, g = 0; r < m; ++r, ++g) {
      if (g == 7) ++g;
      const size_t k = g % d;
      EXPECT(index[r] == g * n + k);
      const size_t L = lens[g * d + k];  // the lost packet's length: its bytes past L recover as zeros
      EXPECT(std::memcmp(out + r * pitch, pkts + (g * d + k) * slot + 6, L - 6) == 0);
    }
  }
  // the device-path pair on a device copy of the assembled batch
  uint8_t *dshards = nullptr, *dout = nullptr;
  uint64_t* dpres = nullptr;
  uint32_t *dlist = nullptr, *dcount = nullptr, *dstats = nullptr;
  uint8_t* dring = nullptr;
  uint16_t* drlens = nullptr;
  EXPECT(hipMalloc(&dshards, n * G * pitch) == hipSuccess && hipMalloc(&dout, G * p * pitch) == hipSuccess &&
         hipMalloc(&dpres, G * 8) == hipSuccess && hipMalloc(&dlist, G * 4) == hipSuccess &&
         hipMalloc(&dcount, 4) == hipSuccess && hipMalloc(&dstats, 20) == hipSuccess &&
         hipMalloc(&dring, keep.size() * slot) == hipSuccess && hipMalloc(&drlens, keep.size() * 2) == hipSuccess);
  EXPECT(hipMemcpy(dring, ring, keep.size() * slot, hipMemcpyHostToDevice) == hipSuccess &&
         hipMemcpy(drlens, rlens, keep.size() * 2, hipMemcpyHostToDevice) == hipSuccess &&
         hipMemset(dpres, 0, G * 8) == hipSuccess);
  uint8_t* dpad = nullptr;
  EXPECT(hipMalloc(&dpad, slot) == hipSuccess && hipMemcpy(dpad, pad, slot, hipMemcpyHostToDevice) == hipSuccess);
  EXPECT(ugo_fec_rx_assemble(ctx, dring, slot, drlens, keep.size(), dpad, 0, G, dshards, S, G * pitch, pitch, dpres,
                             dstats, nullptr) == UGO_FEC_OK);
  EXPECT(ugo_fec_lossy_groups(ctx, dpres, G, UGO_FEC_RECONSTRUCT_DATA_ONLY, dlist, dcount, nullptr) == UGO_FEC_OK);
  EXPECT(ugo_fec_reconstruct_list(ctx, dshards, dpres, G, dlist, dcount, G, S, G * pitch, pitch, dout, pitch, p * pitch,
                                  UGO_FEC_RECONSTRUCT_DATA_ONLY, nullptr, nullptr) == UGO_FEC_OK);
  EXPECT(hipDeviceSynchronize() == hipSuccess);
  uint32_t cnt = 0;
  EXPECT(hipMemcpy(&cnt, dcount, 4, hipMemcpyDeviceToHost) == hipSuccess);
  EXPECT(cnt == G);  // every group has a lost data row (group 7 listed, with no output)
  // round 6: the same ring into frame rows (64-B pitch), its payload columns equal the payload rows'
  {
    const size_t fp = 1536;
    uint8_t* fsh = nullptr;
    uint64_t* fpres = nullptr;
    EXPECT(hipMalloc(&fsh, n * G * fp) == hipSuccess && hipMalloc(&fpres, G * 8) == hipSuccess &&
           hipMemset(fpres, 0, G * 8) == hipSuccess);
    EXPECT(ugo_fec_rx_assemble_frames(ctx, dring, slot, drlens, keep.size(), dpad, 0, G, fsh, S, G * fp, fp, fpres,
                                      nullptr, nullptr) == UGO_FEC_OK);
    EXPECT(hipDeviceSynchronize() == hipSuccess);
    std::vector<uint8_t> a(n * G * pitch), b(n * G * fp);
    std::vector<uint64_t> pa(G), pb(G);
    EXPECT(hipMemcpy(a.data(), dshards, a.size(), hipMemcpyDeviceToHost) == hipSuccess &&
           hipMemcpy(b.data(), fsh, b.size(), hipMemcpyDeviceToHost) == hipSuccess &&
           hipMemcpy(pa.data(), dpres, G * 8, hipMemcpyDeviceToHost) == hipSuccess &&
           hipMemcpy(pb.data(), fpres, G * 8, hipMemcpyDeviceToHost) == hipSuccess);
    EXPECT(pa == pb);
    for (size_t g = 0; g < G; ++g)
      for (size_t r = 0; r < n; ++r)
        if ((pa[g] >> r) & 1) {  // a placed row (the list reconstruct above rebuilt none in place)
          EXPECT(std::memcmp(&a[r * G * pitch + g * pitch], &b[r * G * fp + g * fp + 6], S) == 0);
        }
    (void)hipFree(fsh);
    (void)hipFree(fpres);
  }
  for (void* q : {static_cast<void*>(dshards), static_cast<void*>(dout), static_cast<void*>(dpres),
                  static_cast<void*>(dlist), static_cast<void*>(dcount), static_cast<void*>(dstats),
                  static_cast<void*>(dring), static_cast<void*>(drlens), static_cast<void*>(dpad)})
    (void)hipFree(q);
  for (void* v : owned) {
    if (pinned)
      ugo_fec_host_free(v);
    else
      std::free(v);
  }
  ugo_fec_destroy(ctx);
}

// the per-call service's failure paths (round 4): a forced stall past the
// watchdog timeout (the block leaves within the grace period: ERR_HIP, later
// calls on the launch path), a restart, and a block that never leaves within
// the grace period (poisoned context: every call fails, destroy leaks what the
// block reads -- the stage stays allocated here until the block is done)
void service_watchdog() {
  const int d = 10, p = 3, n = d + p;
  const size_t S = 1470, pitch = 1472;
  uint8_t* g = nullptr;
  EXPECT(ugo_fec_host_alloc(n * pitch, reinterpret_cast<void**>(&g)) == UGO_FEC_OK);
  if (!g) return;
  for (size_t i = 0; i < n * pitch; ++i) g[i] = rb();
  std::vector<uint8_t> want(g, g + n * pitch);
  ugo_fec* ref = nullptr;
  EXPECT(ugo_fec_create(0, d, p, &ref) == UGO_FEC_OK);
  EXPECT(ugo_fec_encode_host(ref, want.data(), 1, S, pitch) == UGO_FEC_OK);  // pageable: staged path
  ugo_fec_destroy(ref);
  ugo_fec* ctx = nullptr;
  EXPECT(ugo_fec_create(0, d, p, &ctx) == UGO_FEC_OK);
  EXPECT(ugo_fec_service_config(ctx, 50, 5000, 300000) == UGO_FEC_OK);
  EXPECT(ugo_fec_service_start(ctx, 1000000) == UGO_FEC_OK);
  EXPECT(ugo_fec_encode_host(ctx, g, 1, S, pitch) == UGO_FEC_ERR_HIP);  // timed out, block gone
  EXPECT(ugo_fec_poisoned(ctx) == 0);
  EXPECT(std::memcmp(g, want.data(), n * pitch) == 0);
  EXPECT(ugo_fec_encode_host(ctx, g, 1, S, pitch) == UGO_FEC_OK);  // launch path
  EXPECT(ugo_fec_service_config(ctx, 0, 0, 0) == UGO_FEC_OK);
  EXPECT(ugo_fec_service_start(ctx, 1000000) == UGO_FEC_OK);
  for (int i = 0; i < 20; ++i) {  // served; stop / start while the block is resident
    EXPECT(ugo_fec_encode_host(ctx, g, 1, S, pitch) == UGO_FEC_OK);
    if (i % 5 == 4) {
      EXPECT(ugo_fec_service_stop(ctx) == UGO_FEC_OK);
      EXPECT(ugo_fec_service_start(ctx, 1000000) == UGO_FEC_OK);
    }
  }
  EXPECT(std::memcmp(g, want.data(), n * pitch) == 0);
  ugo_fec_destroy(ctx);
  // poisoned: stall 1.2 s, timeout 50 ms, grace 100 ms
  ctx = nullptr;
  EXPECT(ugo_fec_create(0, d, p, &ctx) == UGO_FEC_OK);
  EXPECT(ugo_fec_service_config(ctx, 50, 100, 1200000) == UGO_FEC_OK);
  EXPECT(ugo_fec_service_start(ctx, 1000000) == UGO_FEC_OK);
  EXPECT(ugo_fec_encode_host(ctx, g, 1, S, pitch) == UGO_FEC_ERR_HIP);
  EXPECT(ugo_fec_poisoned(ctx) == 1);
  EXPECT(ugo_fec_encode_host(ctx, g, 1, S, pitch) == UGO_FEC_ERR_HIP);
  EXPECT(ugo_fec_service_start(ctx, 0) == UGO_FEC_ERR_HIP);
  ugo_fec_destroy(ctx);  // leaks the mailbox and tables the block still reads
  EXPECT(hipDeviceSynchronize() == hipSuccess);  // the stalled block serves, sees the stop line, leaves
  EXPECT(std::memcmp(g, want.data(), n * pitch) == 0);
  ugo_fec_host_free(g);
}

// set_batch whose pinned batch cannot be allocated (ugo_fec_set_host_alloc_limit):
// ERR_HIP, per-call mode, and input keeps working
void fec_object_alloc_failure() {
  ugo_fecconn* f = nullptr;
  EXPECT(ugo_fecconn_new(64, 10, 3, 0, &f) == UGO_FEC_OK);
  if (!f) return;
  std::vector<uint8_t> out(64 * 10 * 1476);
  int nrec = 0;
  size_t rl = 0;
  EXPECT(ugo_fecconn_set_batch(f, 4, out.data(), out.size(), &nrec, &rl) == UGO_FEC_OK);
  ugo_fec_set_host_alloc_limit(4096);
  EXPECT(ugo_fecconn_set_batch(f, 8, out.data(), out.size(), &nrec, &rl) == UGO_FEC_ERR_HIP);
  ugo_fec_set_host_alloc_limit(0);
  // one lossy group (data shard 2 lost) through input, per call now
  std::vector<std::vector<uint8_t>> grp(13, std::vector<uint8_t>(1476));
  std::vector<uint8_t*> ptr(13);
  std::vector<size_t> lens(13, 1476);
  for (int k = 0; k < 13; ++k) {
    for (auto& b : grp[k]) b = rb();
    ptr[k] = grp[k].data();
  }
  for (int k = 0; k < 10; ++k) EXPECT(ugo_fecconn_mark_data(f, grp[k].data()) == UGO_FEC_OK);
  EXPECT(ugo_fecconn_calc_ecc(f, ptr.data(), lens.data(), 13, 6, 1476) == UGO_FEC_OK);
  for (int k = 10; k < 13; ++k) EXPECT(ugo_fecconn_mark_fec(f, grp[k].data()) == UGO_FEC_OK);
  int got = 0;
  for (int k = 0; k < 13; ++k) {
    if (k == 2) continue;
    uint32_t sq = 0;
    uint16_t fl = 0;
    EXPECT(ugo_fecconn_input(f, grp[k].data(), 1476, &sq, &fl, out.data(), out.size(), &nrec, &rl) == UGO_FEC_OK);
    got += nrec;
  }
  EXPECT(got == 1 && std::memcmp(out.data(), grp[2].data() + 6, 1470) == 0);
  ugo_fecconn_free(f);
}

}  // namespace

int main() {
  check_shards_cases();
  null_args();
  for (bool pinned : {true, false}) {
    host_round_trip(10, 3, 1350, 300, pinned);
    host_round_trip(10, 3, 1470, 1, pinned);
    host_round_trip(4, 2, 77, 7, pinned);
    host_round_trip(32, 8, 9000, 12, pinned);
    host_round_trip(20, 9, 1100, 33, pinned);
    host_round_trip_wide(70, 10, 64, 5, pinned);
    host_round_trip_wide(8, 120, 48, 3, pinned);
  }
  host_round_trip(10, 3, 1470, 1, true, true);
  host_round_trip(10, 3, 1476, 16, true, true);
  host_round_trip(4, 2, 77, 7, true, true);
  fec_object(1);
  fec_object(16);
  fec_object(3, UGO_FECCONN_BATCH_OVERLAP);
  fec_object(16, UGO_FECCONN_BATCH_OVERLAP);
  fec_object(4, 0, true);
  tx_rx_batch();
  host_rx_tx_paths(true);
  host_rx_tx_paths(false);
  fec_object_alloc_failure();
  service_watchdog();
  std::printf("{\"asan_driver\": \"%s\", \"failures\": %d}\n", failures ? "FAIL" : "ok", failures);
  return failures ? 1 : 0;
}
