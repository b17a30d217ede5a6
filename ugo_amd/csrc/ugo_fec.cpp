// ugo_fec.cpp -- C-ABI (include/ugo_fec.h) of the MI355X FEC engine.
//
// Host-side control plane only: geometry validation (reedsolomon.New as called
// at ugo/fec.go:59), the code matrix, the decode-descriptor table (the analogue
// of klauspost's inversion-tree cache, built once per context instead of per
// erasure pattern on first use), argument checks mirroring checkShards, and
// launch selection.  All byte arithmetic runs in the gfx950 kernels of
// fec_kernels.hip; there is no CPU compute path for shard bytes.
#include "../../include/ugo_fec.h"

#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

#include "fec_kernels.hpp"
#include "gf256.hpp"
#include "host/rc4.hpp"
#include "launch.hpp"
#include "rx_kernels.hpp"
#include "tx_kernels.hpp"
#include "pkt_kernels.hpp"

namespace {

constexpr int kStreams = 3;
constexpr size_t kStageBytes = size_t(64) << 20;  // per host-path staging buffer
// RX ring stages in flight: with two, both stages' copies ran at once and the
// next pair waited for the first stage's assembly -- the link idled ~0.15 ms
// per 2.4-ms pair (profiles/r5/host_rx_trace); with four a copy stream always
// has its next stage free.
constexpr int kRxStages = 4;
constexpr size_t kZeroCopyEncodeBytes = size_t(4) << 20;  // pinned encode batches up to this run zero-copy
constexpr uint32_t kMaxItems = 0x7fffffffu;

inline size_t round_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

// Groups per launch: a launch's work-item count is a uint32.  The vector
// kernels may pad every group to a whole number of waves (k_apply_qa: rows
// rounded up to 64 chunks), so a slice is sized from the padded count --
// otherwise a short-row code (e.g. 1 chunk per row, padded to 64) would wrap
// groups * 64 past 2^32 and leave most of the slice unwritten.
inline size_t slice_groups(uint32_t chunks, bool fast) {
  const size_t per_group = fast ? round_up(chunks, 64) : chunks;
  return std::max<size_t>(1, kMaxItems / per_group);
}

struct DeviceGuard {
  int prev = -1;
  bool ok = true;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) ok = hipSetDevice(dev) == hipSuccess;
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

}  // namespace

struct ugo_fec {
  int device = 0;
  int d = 0, p = 0, n = 0;
  std::vector<uint8_t> M;  // n x d
  uint32_t dpad = 0, epad = 0, desc_stride = 0;
  int table_max = 16;       // d+p <= table_max -> host-built pattern table (MODE 1)
  uint8_t* d_M = nullptr;
  uint8_t* d_gf = nullptr;  // exp[512] | log[256] | pad | gf::perm_tables at +1024
  uint8_t* d_encdesc = nullptr;
  uint8_t* d_table = nullptr;
  // stream-ordered scratch (MODE 2 descriptors, RX claim words): allocated and
  // freed on the call's own stream, so calls on different streams never share
  // a workspace
  hipMemPool_t pool = nullptr;
  std::vector<std::pair<hipStream_t, hipEvent_t>> scratch_ev;  // per stream: behind its last scratch free
  // host-path staging
  hipStream_t streams[kStreams] = {};
  uint8_t* d_stage[kStreams] = {};
  uint64_t* d_mask[kStreams] = {};
  int8_t* d_status[kStreams] = {};
  uint64_t* d_zc_mask = nullptr;  // zero-copy host reconstruct: presence masks / status of the batch,
  int8_t* d_zc_status = nullptr;   // pinned host memory the kernels read / write through its mapping
  // RX: k_rx_begin's record of calls that found a presence bit set (atomicMax of
  // the call id), and this context's call counter
  unsigned long long* d_rxseen = nullptr;
  unsigned long long rx_calls = 0;
  // one-launch lossy list (k_lossy_list1): per stream, the tiles' epoch-tagged
  // count words (context-owned, zeroed once) and that stream's call epoch
  struct LossyWords {
    hipStream_t s;
    uint64_t* words;
    size_t tiles;
    uint32_t epoch;
  };
  std::vector<LossyWords> lossy_words;
  size_t zc_groups = 0;
  // d+p > 64: decode descriptors built on the host, one per erasure pattern
  // (klauspost caches its inversions per pattern the same way)
  std::unordered_map<std::string, std::vector<uint8_t>> wide_cache;
  int tx_route = 0;  // host TX wire route (ugo_fec_set_tx_host_route): 0 D2H copy, 1 mapped write
#ifndef UGO_COPY_QUEUE_DEFAULT
#define UGO_COPY_QUEUE_DEFAULT 1
#endif
  bool host_copy_queue = UGO_COPY_QUEUE_DEFAULT != 0;  // ugo_fec_set_host_copy_queue: streams[1] low priority
  bool streams_shared = false;  // streams[1] is the process-wide low-priority copy stream (not ours to destroy)
  size_t stage_groups = 0;  // groups per staging buffer
  size_t stage_pitch = 0;
  // launch timing (ugo_fec_timing_begin/end)
  bool timing = false;
  ugo::kern::LaunchTimer timer;
  // per-call service (ugo_fec_service_start): mailbox in coherent pinned memory
  bool svc_on = false;
  uint64_t svc_idle_ticks = 0;
  ugo::kern::SvcBox* svc_box = nullptr;   // host address
  ugo::kern::SvcBox* svc_dbox = nullptr;  // device view
  hipStream_t svc_stream = nullptr;
  uint32_t svc_seq = 0;                 // the last seq posted on the mailbox line
  uint32_t svc_timeout_ms = 5000;       // watchdog: a call's wait for an answer
  uint32_t svc_grace_ms = 5000;         // then: the wait for the block to leave
  uint32_t svc_stall_us = 0;            // tests only (ugo_fec_service_config)
  uint64_t svc_khz = 100000;            // wall_clock64's rate (100 MHz on gfx950)
  // the service block did not leave within the grace period: it may still read
  // the mailbox and tables and write a caller's batch, so every call fails and
  // destroy leaks what the block reads
  bool poisoned = false;
};

namespace {

// Makes the context's launch timer (if on) the one the launchers of this
// thread see, for the duration of one ABI call.
struct TimerScope {
  ugo::kern::LaunchTimer* prev;
  explicit TimerScope(ugo_fec* c) : prev(ugo::kern::current_timer()) {
    ugo::kern::current_timer() = (c && c->timing) ? &c->timer : nullptr;
  }
  ~TimerScope() { ugo::kern::current_timer() = prev; }
};

void timer_release(ugo_fec* c) {
  ugo::kern::LaunchTimer& t = c->timer;
  for (size_t i = 0; i < 2 * t.cap; ++i)
    if (t.ev[i]) (void)hipEventDestroy(t.ev[i]);
  delete[] t.ev;
  delete[] t.kid;
  t = ugo::kern::LaunchTimer{};
  c->timing = false;
}

// Decode descriptor for one presence mask (layout: fec_kernels.hip).
// Survivors = first d present rows in index order (klauspost Reconstruct),
// outputs = erased data rows then erased parity rows, coefficients
// Dinv[r] (data row r) or M[r] * Dinv (parity row r).
// Presence words per group: one for d+p <= 64, ceil((d+p)/64) above (bit r of
// the pattern = bit r % 64 of word r / 64).
size_t mask_words(const ugo_fec* c) { return (size_t(c->n) + 63) / 64; }

int build_desc_bits(const ugo_fec* c, const uint64_t* w, uint8_t* out) {
  const int d = c->d, n = c->n;
  auto present = [w](int r) { return (w[r >> 6] >> (r & 63)) & 1; };
  std::memset(out, 0, c->desc_stride);
  int np = 0;
  for (int r = 0; r < n; ++r) np += present(r);
  if (np == n) return UGO_FEC_OK;  // e = 0: nothing to rebuild
  if (np < d) {
    out[2] = UGO_FEC_ERR_TOO_FEW_SHARDS;
    return UGO_FEC_OK;
  }
  std::vector<uint8_t> sub(size_t(d) * d), inv(size_t(d) * d), work(size_t(2) * d * d);
  std::vector<int> surv, outr;
  for (int r = 0; r < n; ++r) {
    if (present(r)) {
      if (int(surv.size()) < d) surv.push_back(r);
    } else {
      outr.push_back(r);
    }
  }
  for (int i = 0; i < d; ++i) std::memcpy(&sub[size_t(i) * d], &c->M[size_t(surv[i]) * d], d);
  if (!ugo::gf::invert(d, sub.data(), inv.data(), work.data())) {
    out[2] = UGO_FEC_ERR_SINGULAR;
    return UGO_FEC_ERR_SINGULAR;
  }
  int e_data = 0;
  for (int r : outr) e_data += r < d;
  out[0] = static_cast<uint8_t>(outr.size());
  out[1] = static_cast<uint8_t>(e_data);
  for (int i = 0; i < d; ++i) out[4 + i] = static_cast<uint8_t>(surv[i]);
  for (size_t i = 0; i < outr.size(); ++i) out[4 + c->dpad + i] = static_cast<uint8_t>(outr[i]);
  uint8_t* coef = out + 4 + c->dpad + c->epad;
  for (size_t i = 0; i < outr.size(); ++i) {
    const int r = outr[i];
    for (int k = 0; k < d; ++k) {
      uint8_t v;
      if (r < d) {
        v = inv[size_t(r) * d + k];
      } else {
        v = 0;
        for (int j = 0; j < d; ++j) v ^= ugo::gf::mul(c->M[size_t(r) * d + j], inv[size_t(j) * d + k]);
      }
      coef[i * c->dpad + k] = v;
    }
  }
  return UGO_FEC_OK;
}

int build_desc(const ugo_fec* c, uint64_t mask, uint8_t* out) { return build_desc_bits(c, &mask, out); }

int hip_status(hipError_t e) { return e == hipSuccess ? UGO_FEC_OK : UGO_FEC_ERR_HIP; }

int svc_stop(ugo_fec* c);
bool is_shared_stream(const ugo_fec* c, int i);

void free_ctx(ugo_fec* c) {
  if (!c) return;
  DeviceGuard g(c->device);
  // the resident block leaves before its mailbox and tables go
  if (c->poisoned || svc_stop(c) != UGO_FEC_OK) {
    // poisoned: a block that never left may still read the mailbox and tables
    // and write a caller's batch.  Every device-side release -- hipFree,
    // hipHostFree, stream and pool destruction -- synchronizes with the device
    // and would wait for that block (forever, if it never leaves), so all of
    // it is leaked; only the host-side object goes.
    delete c;
    return;
  }
  (void)hipHostFree(c->svc_box);
  (void)hipFree(c->d_M);
  (void)hipFree(c->d_gf);
  (void)hipFree(c->d_encdesc);
  (void)hipFree(c->d_table);
  (void)hipFree(c->d_rxseen);
  for (auto& lw : c->lossy_words) (void)hipFree(lw.words);
  timer_release(c);
  (void)hipHostFree(c->d_zc_mask);
  (void)hipHostFree(c->d_zc_status);
  for (int i = 0; i < kStreams; ++i) {
    (void)hipFree(c->d_stage[i]);
    (void)hipFree(c->d_mask[i]);
    (void)hipFree(c->d_status[i]);
    if (c->streams[i] && !is_shared_stream(c, i)) (void)hipStreamDestroy(c->streams[i]);
  }
  // this context's async scratch frees still queued on the callers' streams
  for (auto& se : c->scratch_ev) {
    (void)hipEventSynchronize(se.second);
    (void)hipEventDestroy(se.second);
  }
  if (c->pool) (void)hipMemPoolDestroy(c->pool);
  delete c;
}

struct Layout {
  uint64_t rstride;  // bytes between rows of one group
  uint64_t gstride;  // bytes between groups
};

Layout interleaved(const ugo_fec* c, size_t pitch) { return Layout{pitch, uint64_t(c->n) * pitch}; }

// The 16-B vector kernels need aligned rows; every d runs on them (d <= 32:
// register-array kernels, d > 32: the streaming kernels, which take any row
// length and output count).  Unaligned layouts run the byte kernel.
bool fast_layout(const ugo_fec*, const uint8_t* shards, const Layout& L, size_t) {
  return (reinterpret_cast<uintptr_t>(shards) % 16 == 0) && (L.rstride % 16 == 0) && (L.gstride % 16 == 0);
}

// Separate output batch of a reconstruct (ugo_fec_reconstruct_into); none = in place.
struct OutBatch {
  uint8_t* base = nullptr;
  Layout L{0, 0};
};

ugo::kern::Batch base_batch(const ugo_fec* c, uint8_t* shards, size_t S, const Layout& L) {
  ugo::kern::Batch a{};
  a.base = shards;
  a.gstride = L.gstride;
  a.rstride = L.rstride;
  a.nmask = c->n >= 64 ? ~0ull : ((1ull << c->n) - 1);
  a.S = static_cast<uint32_t>(S);
  a.desc_stride = c->desc_stride;
  a.d = static_cast<uint32_t>(c->d);
  a.dpad = c->dpad;
  a.epad = c->epad;
  a.mult = reinterpret_cast<const uint32_t*>(c->d_gf + 1024);
  return a;
}

// Bytes spanned by `rows` x `groups` slots of S bytes (row r of group g at
// g*gstride + r*rstride).
size_t extent(size_t S, size_t rstride, size_t rows, size_t gstride, size_t groups) {
  if (rows == 0 || groups == 0) return 0;
  return (groups - 1) * gstride + (rows - 1) * rstride + S;
}

// True if those slots are pairwise disjoint: sorted by stride, the smaller
// stride is >= S and the larger one clears a whole run of the smaller.
bool layout_disjoint(size_t S, size_t rstride, size_t rows, size_t gstride, size_t groups) {
  size_t small = rstride, ns = rows, large = gstride, nl = groups;
  if (ns <= 1 || (nl > 1 && gstride < rstride)) {
    std::swap(small, large);
    std::swap(ns, nl);
  }
  if (ns > 1 && small < S) return false;
  if (nl > 1 && large < (ns - 1) * small + S) return false;
  return true;
}

int check_batch(const ugo_fec* c, const void* shards, size_t groups, size_t S, const Layout& L) {
  if (!c) return UGO_FEC_ERR_INVALID_ARG;
  if (c->poisoned) return UGO_FEC_ERR_HIP;  // a service block that never left (svc_retire)
  if (S == 0) return UGO_FEC_ERR_SHARD_NO_DATA;  // checkShards: all shards empty
  if (S > 0xffffffffu) return UGO_FEC_ERR_INVALID_ARG;
  if (groups == 0) return UGO_FEC_OK;  // an empty batch has no layout to check
  // no two shard slots may overlap: kernels write rows other lanes read
  if (!layout_disjoint(S, L.rstride, size_t(c->n), L.gstride, groups)) return UGO_FEC_ERR_INVALID_ARG;
  if (groups && !shards) return UGO_FEC_ERR_INVALID_ARG;
  return UGO_FEC_OK;
}

// Dense planar batch: groups packed back to back in each row (group stride ==
// S, no padding), rows 16-B aligned.  Encode is column-wise and every group
// uses the same matrix, so k = 16 / gcd(S, 16) consecutive groups form one
// pseudo-group of k*S bytes, a whole number of 16-B chunks: the vector kernels
// then read and write exactly the batch's bytes, with no padding and no
// partial chunk except at the batch's end.
bool dense_rows(const uint8_t* shards, size_t S, const Layout& L) {
  return L.gstride == S && S % 16 != 0 && reinterpret_cast<uintptr_t>(shards) % 16 == 0 && L.rstride % 16 == 0 &&
         S <= 0xffffffffu / 16;
}

int encode_dev(ugo_fec* c, uint8_t* shards, size_t groups, size_t S, const Layout& L, hipStream_t s) {
  if (c->p == 0 || groups == 0) return UGO_FEC_OK;
  if (groups > 1 && dense_rows(shards, S, L)) {
    size_t k = 16;
    while (S % (16 / k * 2) == 0) k /= 2;  // k = 16 / gcd(S, 16)
    const size_t full = groups / k, tail = groups % k;
    int st = full ? encode_dev(c, shards, full, k * S, Layout{L.rstride, k * S}, s) : UGO_FEC_OK;
    if (st == UGO_FEC_OK && tail)  // one pseudo-group (its group stride is never used)
      st = encode_dev(c, shards + full * k * S, 1, tail * S, Layout{L.rstride, round_up(tail * S, 16)}, s);
    return st;
  }
  const bool fast = fast_layout(c, shards, L, S);
  ugo::kern::Batch a = base_batch(c, shards, S, L);
  a.desc = c->d_encdesc;
  a.chunks = static_cast<uint32_t>(fast ? (S + 15) / 16 : (S + 3) / 4);
  const size_t per = slice_groups(a.chunks, fast);
  for (size_t g0 = 0; g0 < groups; g0 += per) {
    const size_t gn = std::min(per, groups - g0);
    a.g0 = g0;
    a.items = static_cast<uint32_t>(gn * a.chunks);
    hipError_t e;
    if (fast && ugo::kern::has_const_encode(c->d, c->p))
      e = ugo::kern::launch_encode_const(c->d, c->p, a, s);
    else if (fast)
      e = ugo::kern::launch_apply(0, ugo::kern::apply_dmax(c->d), a, s);
    else
      e = ugo::kern::launch_apply_bytes(0, a, s);
    if (e != hipSuccess) return UGO_FEC_ERR_HIP;
  }
  return UGO_FEC_OK;
}

// Scratch of `bytes` on stream s, from the context's memory pool (created on
// first use; memory is kept in the pool between calls, so after the first call
// an allocation is a host-side bookkeeping step).  Free with scratch_free on
// the same stream.
int scratch_alloc(ugo_fec* c, size_t bytes, hipStream_t s, void** out) {
  *out = nullptr;
  if (!c->pool) {
    hipMemPoolProps props{};
    props.allocType = hipMemAllocationTypePinned;
    props.location.type = hipMemLocationTypeDevice;
    props.location.id = c->device;
    if (hipMemPoolCreate(&c->pool, &props) != hipSuccess) {
      c->pool = nullptr;
      return UGO_FEC_ERR_HIP;
    }
    uint64_t keep = ~0ull;
    (void)hipMemPoolSetAttribute(c->pool, hipMemPoolAttrReleaseThreshold, &keep);
  }
  return hip_status(hipMallocFromPoolAsync(out, bytes ? bytes : 16, c->pool, s));
}

// Frees scratch on its stream and records, per stream, an event behind the
// free: destroying the context waits for exactly those events (its own
// scratch frees), not for every stream on the device -- other contexts'
// in-flight batches do not stall a destroy.
int scratch_free(ugo_fec* c, void* ptr, hipStream_t s) {
  if (!ptr) return UGO_FEC_OK;
  if (hipFreeAsync(ptr, s) != hipSuccess) return UGO_FEC_ERR_HIP;
  hipEvent_t ev = nullptr;
  for (auto& se : c->scratch_ev)
    if (se.first == s) ev = se.second;
  if (!ev) {
    if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) return UGO_FEC_ERR_HIP;
    c->scratch_ev.emplace_back(s, ev);
  }
  return hip_status(hipEventRecord(ev, s));
}

bool fast_out(const OutBatch& O) {
  return !O.base || (reinterpret_cast<uintptr_t>(O.base) % 16 == 0 && O.L.rstride % 16 == 0 && O.L.gstride % 16 == 0);
}

constexpr size_t kWideCacheMax = 4096;  // patterns kept per context (d+p > 64)

// d+p > 64 (wider than one presence word): the decode descriptors are built on
// the host per erasure pattern (cached) and uploaded; the apply kernels run as
// for k_prepare's descriptors (MODE 2).  The masks are read on the host: from
// host_present when the caller has them there, else copied from the device
// (a synchronising copy -- wide codes are not ugo's geometry).
int reconstruct_wide(ugo_fec* c, uint8_t* shards, const uint64_t* present, size_t groups, size_t S,
                     const Layout& L, unsigned flags, int8_t* status, hipStream_t s, const OutBatch& O,
                     const uint64_t* host_present) {
  const size_t W = mask_words(c);
  std::vector<uint64_t> hm;
  if (!host_present) {
    hm.resize(groups * W);
    if (hipMemcpyAsync(hm.data(), present, hm.size() * sizeof(uint64_t), hipMemcpyDefault, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
      return UGO_FEC_ERR_HIP;
    host_present = hm.data();
  }
  const bool fast = fast_layout(c, shards, L, S) && fast_out(O);
  ugo::kern::Batch a = base_batch(c, shards, S, L);
  a.out = O.base;
  a.ogstride = O.L.gstride;
  a.orstride = O.L.rstride;
  a.status = status;
  a.data_only = (flags & UGO_FEC_RECONSTRUCT_DATA_ONLY) ? 1u : 0u;
  a.chunks = static_cast<uint32_t>(fast ? (S + 15) / 16 : (S + 3) / 4);
  const size_t per = std::min<size_t>(slice_groups(a.chunks, fast), 65536);
  const size_t stride = c->desc_stride;
  std::vector<uint8_t> hd(std::min(per, groups) * stride);
  uint8_t* work = nullptr;
  int st = scratch_alloc(c, hd.size() + 64, s, reinterpret_cast<void**>(&work));
  if (st) return st;
  struct Release {
    ugo_fec* c;
    uint8_t* p;
    hipStream_t s;
    ~Release() { (void)scratch_free(c, p, s); }
  } release{c, work, s};
  for (size_t g0 = 0; g0 < groups; g0 += per) {
    const size_t gn = std::min(per, groups - g0);
    for (size_t g = 0; g < gn; ++g) {
      const uint64_t* w = host_present + (g0 + g) * W;
      std::string key(reinterpret_cast<const char*>(w), W * sizeof(uint64_t));
      auto it = c->wide_cache.find(key);
      if (it == c->wide_cache.end()) {
        std::vector<uint8_t> dsc(stride);
        (void)build_desc_bits(c, w, dsc.data());  // a failure is the group's status byte
        if (c->wide_cache.size() >= kWideCacheMax) c->wide_cache.clear();
        it = c->wide_cache.emplace(std::move(key), std::move(dsc)).first;
      }
      std::memcpy(&hd[g * stride], it->second.data(), stride);
    }
    // hd is refilled for the next slice: the copy must have read it first
    if (hipMemcpyAsync(work, hd.data(), gn * stride, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
      return UGO_FEC_ERR_HIP;
    a.g0 = g0;
    a.items = static_cast<uint32_t>(gn * a.chunks);
    a.desc = work;
    a.g_desc0 = g0;
    const hipError_t e = fast ? ugo::kern::launch_apply(2, ugo::kern::apply_dmax(c->d), a, s)
                              : ugo::kern::launch_apply_bytes(2, a, s);
    if (e != hipSuccess) return UGO_FEC_ERR_HIP;
  }
  return UGO_FEC_OK;
}

int reconstruct_dev(ugo_fec* c, uint8_t* shards, const uint64_t* present, size_t groups, size_t S,
                    const Layout& L, unsigned flags, int8_t* status, hipStream_t s, const OutBatch& O = {},
                    const uint64_t* host_present = nullptr) {
  if (groups == 0) return UGO_FEC_OK;
  if (!present) return UGO_FEC_ERR_INVALID_ARG;
  if (c->n > 64) return reconstruct_wide(c, shards, present, groups, S, L, flags, status, s, O, host_present);
  // A dense planar batch (group stride == S) runs k_apply_pd: lanes on the
  // rows' aligned 16-B chunks, the bytes of a chunk that straddles two groups
  // split between two lanes.  That kernel's shape: d <= 16, p <= 4, S >= 1009.
  const bool dense = dense_rows(shards, S, L) && ugo::kern::apply_dmax(c->d) > 0 &&
                     ugo::kern::apply_dmax(c->d) <= 16 && c->epad == 4 && S >= ugo::kern::kDenseMinS;
  const bool fast = (fast_layout(c, shards, L, S) && fast_out(O)) || dense;
  const int mode = c->d_table ? 1 : 2;
  ugo::kern::Batch a = base_batch(c, shards, S, L);
  a.out = O.base;
  a.ogstride = O.L.gstride;
  a.orstride = O.L.rstride;
  a.present = present;
  a.status = status;
  a.data_only = (flags & UGO_FEC_RECONSTRUCT_DATA_ONLY) ? 1u : 0u;
  a.chunks = static_cast<uint32_t>(fast ? (S + 15) / 16 : (S + 3) / 4);
  size_t per = slice_groups(a.chunks, fast);
  if (dense) {  // slices start on 16-B aligned bytes: a multiple of 16 / gcd(S, 16) groups
    per = std::max<size_t>(16, per / 16 * 16);
  }
  uint8_t* work = nullptr;
  if (mode == 2) {
    // per-group descriptors, bounded workspace (<= 64 Ki groups per slice)
    per = std::min<size_t>(per, 65536);
    const int st = scratch_alloc(c, std::min(per, groups) * c->desc_stride + 64, s, reinterpret_cast<void**>(&work));
    if (st) return st;
  }
  struct Release {  // the workspace goes back to the pool after this call's kernels
    ugo_fec* c;
    uint8_t* p;
    hipStream_t s;
    ~Release() { (void)scratch_free(c, p, s); }
  } release{c, work, s};
  for (size_t g0 = 0; g0 < groups; g0 += per) {
    const size_t gn = std::min(per, groups - g0);
    a.g0 = g0;
    a.items = static_cast<uint32_t>(gn * a.chunks);
    if (mode == 1) {
      a.desc = c->d_table;
    } else {
      ugo::kern::Prep pr{};
      pr.desc = work;
      pr.present = present;
      pr.M = c->d_M;
      pr.gf_exp = c->d_gf;
      pr.gf_log = c->d_gf + 512;
      pr.g0 = g0;
      pr.g_desc0 = g0;
      pr.nmask = a.nmask;
      pr.desc_stride = c->desc_stride;
      pr.d = static_cast<uint32_t>(c->d);
      pr.n = static_cast<uint32_t>(c->n);
      pr.dpad = c->dpad;
      pr.epad = c->epad;
      if (ugo::kern::launch_prepare(pr, static_cast<uint32_t>(gn), s) != hipSuccess) return UGO_FEC_ERR_HIP;
      a.desc = work;
      a.g_desc0 = g0;
    }
    hipError_t e;
    if (dense) {
      ugo::kern::Batch b = a;
      b.base = shards + g0 * S;
      b.n = static_cast<uint32_t>(gn);
      b.items = static_cast<uint32_t>((gn * S + 15) / 16);
      e = ugo::kern::launch_apply_dense(mode, ugo::kern::apply_dmax(c->d), b, s);
    } else {
      e = fast ? ugo::kern::launch_apply(mode, ugo::kern::apply_dmax(c->d), a, s)
               : ugo::kern::launch_apply_bytes(mode, a, s);
    }
    if (e != hipSuccess) return UGO_FEC_ERR_HIP;
  }
  return UGO_FEC_OK;
}

// The host paths' streams: 0 kernels (and host TX's D2H copies), 1 H2D copies,
// 2 the staged paths' third stream.  HIP maps a process's streams onto a small
// pool of hardware queues per priority class (GPU_MAX_HW_QUEUES, 4 here), and a
// queue processes its packets in order.  When host TX's H2D stream shared a
// queue with the stream its D2H copies ran on, each D2H copy waited behind the
// next chunk's H2D dependency and the two copy directions ran one after the
// other: 40.5 ms instead of 26.6 for 65,536 (10+3) groups, depending on the
// streams the process had made before (profiles/r5/host_tx_route_ab.md).  So
// stream 1 comes from the low-priority class, a pool of its own (26.5-26.6 ms
// in every history tried; ugo_fec_set_host_copy_queue(ctx, 0) turns it off).
// Round 5 kept it opt-in because concurrent device work ran 33-39 % slower with
// it and a resident service block in one process; the cause was the process's
// hardware-queue count, not this queue (svc_queue_cap: past 8 queues the
// scheduler time-slices), and the library now stays within 8.
// The low-priority copy stream is ONE per device for the whole process, shared
// by every context: HIP gives each new low-priority stream a new hardware queue
// up to GPU_MAX_HW_QUEUES, so per-context streams took the process from 8 to 11
// hardware queues with a handful of contexts (test_process_hw_queue_footprint).
// Contexts that share it serialize their H2D copies on it -- they share the
// PCIe link anyway.  Never destroyed (process lifetime).
hipStream_t shared_copy_stream(int device) {
  static std::mutex mu;
  static std::unordered_map<int, hipStream_t>* streams = new std::unordered_map<int, hipStream_t>();
  std::lock_guard<std::mutex> lk(mu);
  hipStream_t& s = (*streams)[device];
  if (!s) {
    int least = 0, greatest = 0;
    if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess ||
        hipStreamCreateWithPriority(&s, hipStreamNonBlocking, least) != hipSuccess)
      s = nullptr;
  }
  return s;
}

bool is_shared_stream(const ugo_fec* c, int i) { return i == 1 && c->streams[1] && c->streams_shared; }

hipError_t create_stream(ugo_fec* c, int i, hipStream_t* s) {
  if (i == 1 && c->host_copy_queue) {
    *s = shared_copy_stream(c->device);
    c->streams_shared = *s != nullptr;
    return *s ? hipSuccess : hipErrorInvalidValue;
  }
  return hipStreamCreateWithFlags(s, hipStreamNonBlocking);
}

int ensure_streams(ugo_fec* c) {
  for (int i = 0; i < kStreams; ++i)
    if (!c->streams[i] && create_stream(c, i, &c->streams[i]) != hipSuccess) return UGO_FEC_ERR_HIP;
  return UGO_FEC_OK;
}

int ensure_stage(ugo_fec* c, size_t pitch) {
  const size_t gbytes = size_t(c->n) * pitch;
  const size_t want = std::max<size_t>(1, kStageBytes / gbytes);
  // every stream first: ugo_fec_set_host_copy_queue drops streams[1], and a
  // staged call must never fall back to the legacy null stream
  const int se = ensure_streams(c);
  if (se) return se;
  if (c->stage_groups >= want && c->stage_pitch == pitch) return UGO_FEC_OK;
  for (int i = 0; i < kStreams; ++i) {
    (void)hipFree(c->d_stage[i]);
    (void)hipFree(c->d_mask[i]);
    (void)hipFree(c->d_status[i]);
    c->d_stage[i] = nullptr;
    c->d_mask[i] = nullptr;
    c->d_status[i] = nullptr;
  }
  c->stage_groups = 0;
  for (int i = 0; i < kStreams; ++i) {
    if (hipMalloc(&c->d_stage[i], want * gbytes + 16) != hipSuccess) return UGO_FEC_ERR_HIP;
    if (hipMalloc(&c->d_mask[i], want * mask_words(c) * sizeof(uint64_t)) != hipSuccess) return UGO_FEC_ERR_HIP;
    if (hipMalloc(&c->d_status[i], want) != hipSuccess) return UGO_FEC_ERR_HIP;
  }
  c->stage_groups = want;
  c->stage_pitch = pitch;
  return UGO_FEC_OK;
}

// Device view of a buffer a kernel will touch: device (or managed) memory as
// is, pinned host memory through its device mapping (the kernel then reads or
// writes it over PCIe: zero-copy, e.g. a recvmmsg ring), anything else --
// pageable host memory the GPU cannot reach, or another GPU's memory -- rejected
// instead of faulting.  Called under the context's DeviceGuard, so the current
// device is the one the kernels run on.
template <typename T>
bool device_view(T*& p) {
  if (!p) return true;
  hipPointerAttribute_t at{};
  if (hipPointerGetAttributes(&at, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  if (at.type == hipMemoryTypeManaged || at.type == hipMemoryTypeUnified) return true;
  if (at.type == hipMemoryTypeDevice) {
    int cur = -1;
    return hipGetDevice(&cur) == hipSuccess && at.device == cur;
  }
  if (at.type != hipMemoryTypeHost || !at.devicePointer) return false;  // unregistered (pageable) memory
  if (at.devicePointer == at.hostPointer) return true;  // one address for host and device (ROCm)
  auto* base = static_cast<uint8_t*>(at.devicePointer);
  if (at.hostPointer) base += reinterpret_cast<const uint8_t*>(p) - static_cast<const uint8_t*>(at.hostPointer);
  p = reinterpret_cast<T*>(base);
  return true;
}

// Zero-copy reconstruct of a pinned host batch (see host_path).
int host_reconstruct_mapped(ugo_fec* c, uint8_t* mapped, const uint64_t* present, size_t groups, size_t S,
                            size_t pitch, unsigned flags, int8_t* status) {
  if (!c->streams[0] && hipStreamCreateWithFlags(&c->streams[0], hipStreamNonBlocking) != hipSuccess)
    return UGO_FEC_ERR_HIP;
  // masks and statuses live in pinned memory too: no copy launches, so a small
  // batch (the per-group calls, FEC::flush) costs one launch and one sync
  const size_t W = mask_words(c);
  if (c->zc_groups < groups) {
    (void)hipHostFree(c->d_zc_mask);
    (void)hipHostFree(c->d_zc_status);
    c->d_zc_mask = nullptr;
    c->d_zc_status = nullptr;
    c->zc_groups = 0;
    const size_t cap = std::max<size_t>(groups, 256);
    if (hipHostMalloc(&c->d_zc_mask, cap * W * sizeof(uint64_t)) != hipSuccess) return UGO_FEC_ERR_HIP;
    if (hipHostMalloc(&c->d_zc_status, cap) != hipSuccess) return UGO_FEC_ERR_HIP;
    c->zc_groups = cap;
  }
  uint64_t* dmask = c->d_zc_mask;
  int8_t* dstatus = c->d_zc_status;
  if (!device_view(dmask) || !device_view(dstatus)) return UGO_FEC_ERR_HIP;
  hipStream_t s = c->streams[0];
  std::memcpy(c->d_zc_mask, present, groups * W * sizeof(uint64_t));
  const int st = reconstruct_dev(c, mapped, dmask, groups, S, interleaved(c, pitch), flags, dstatus, s, {}, present);
  if (st) return st;
  if (hipStreamSynchronize(s) != hipSuccess) return UGO_FEC_ERR_HIP;
  int first = UGO_FEC_OK;
  for (size_t g = 0; g < groups; ++g) {
    const int8_t v = c->d_zc_status[g];
    if (status) status[g] = v;
    if (v && !first) first = v;
  }
  return first;
}

// ---------------------------------------------------------------- per-call service
// The resident k_service block (fec_kernels.hip) serves small pinned batches
// from the context's mailbox: the host fills the request, bumps seq and spins
// on done; a block that has left (idle, alive == 0) is relaunched on the
// service stream, which also orders it after its predecessor.
//
// The line always holds the LAST request posted (c->svc_seq); a block is
// launched with start_seq = the one seq it must not serve: c->svc_seq when no
// request is waiting (that line was served, or abandoned by a stop or a
// timeout), sq - 1 when request sq is posted and waiting.
template <typename T>
T svc_ld(const T& v) { return __atomic_load_n(&v, __ATOMIC_ACQUIRE); }

inline void svc_relax() {  // one spin of the host's wait on the mailbox
#if defined(__x86_64__) || defined(__i386__)
  __builtin_ia32_pause();
#else
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
#endif
}
template <typename T>
void svc_st(T& v, T x) { __atomic_store_n(&v, x, __ATOMIC_RELEASE); }

int svc_launch(ugo_fec* c, uint32_t skip_seq) {
  ugo::kern::SvcArgs sa{};
  sa.a = base_batch(c, nullptr, 0, Layout{0, 0});
  sa.a.desc = c->d_table;
  sa.a.n = static_cast<uint32_t>(c->n);
  sa.encdesc = c->d_encdesc;
  sa.box = c->svc_dbox;
  sa.idle_ticks = c->svc_idle_ticks;
  sa.start_seq = skip_seq;
  sa.stall_ticks = uint64_t(c->svc_stall_us) * c->svc_khz / 1000u;
  svc_st(c->svc_box->alive, 1u);
  if (ugo::kern::launch_service(ugo::kern::apply_dmax(c->d), sa, c->svc_stream) != hipSuccess) {
    svc_st(c->svc_box->alive, 0u);
    c->svc_on = false;  // later calls take the launch path
    return UGO_FEC_ERR_HIP;
  }
  return UGO_FEC_OK;
}

bool svc_eligible(const ugo_fec* c, const uint8_t* mapped, size_t groups, size_t pitch, bool recon) {
  const int dm = ugo::kern::apply_dmax(c->d);
  return c->svc_on && mapped && groups <= size_t(ugo::kern::kSvcMaxGroups) && pitch % 16 == 0 &&
         reinterpret_cast<uintptr_t>(mapped) % 16 == 0 && dm > 0 && dm <= 16 && c->epad == 4 && c->p > 0 &&
         c->desc_stride <= 128 &&
         (!recon || c->d_table);
}

// The service block's stream gets a hardware queue of its own.  HIP spreads
// ordinary streams over a small pool of HSA queues (GPU_MAX_HW_QUEUES, 4 by
// default) and a queue runs its packets in order: an ordinary stream that
// landed on the service's queue would queue every launch and copy behind the
// resident block, i.e. wait out the idle window (tools/svc_sync_probe.cpp:
// a 65,536-group staged host encode took 1002 ms instead of 17 with a 1-s
// window).  Streams of another priority come from another pool, so the
// service runs on a high-priority stream -- but that pool is GPU_MAX_HW_QUEUES
// queues too: a fifth high-priority stream shares a queue with one of the
// first four, and a block resident there would hold back the other's launch
// until the watchdog poisoned it.  So the service streams are a
// process-wide pool per device, at most that many, each leased to ONE context
// while its service is on (the first streams of the priority created in the
// process, so each has its own queue); a context that finds none free serves
// its calls on the launch path (ugo_fec_service_start still succeeds).
#ifndef UGO_SVC_QUEUE
#define UGO_SVC_QUEUE 2
#endif
hipError_t create_service_stream(int device, hipStream_t* out) {
#if UGO_SVC_QUEUE == 1
  // a CU-masked stream is never pooled; but it is a blocking stream
  hipDeviceProp_t prop{};
  hipError_t e = hipGetDeviceProperties(&prop, device);
  if (e != hipSuccess) return e;
  const int cus = std::max(prop.multiProcessorCount, 1);
  std::vector<uint32_t> mask((cus + 31) / 32, 0xffffffffu);
  if (cus % 32) mask.back() = (1u << (cus % 32)) - 1u;
  return hipExtStreamCreateWithCUMask(out, static_cast<uint32_t>(mask.size()), mask.data());
#elif UGO_SVC_QUEUE == 2
  (void)device;
  int lo = 0, hi = 0;
  hipError_t e = hipDeviceGetStreamPriorityRange(&lo, &hi);
  if (e != hipSuccess) return e;
  return hipStreamCreateWithPriority(out, hipStreamNonBlocking, hi);
#else
  (void)device;
  return hipStreamCreateWithFlags(out, hipStreamNonBlocking);
#endif
}

struct SvcStreamPool {
  std::mutex mu;
  std::unordered_map<int, std::vector<hipStream_t>> idle;  // per device: created, not leased
  std::unordered_map<int, int> created;
};

SvcStreamPool& svc_pool() {
  static SvcStreamPool* p = new SvcStreamPool();  // process lifetime: its streams are never destroyed
  return *p;
}

// The process's hardware queues: HIP keeps up to GPU_MAX_HW_QUEUES per
// priority class (4 by default).  Past 8 queues in one process the GPU's
// scheduler runs them oversubscribed (time-sliced), and with a service block
// resident -- a queue that never idles -- concurrent work in the process ran
// 32-33 % slower, whatever the queues were: 8 normal + 1 high, or 4 normal +
// 4 high + 1 low; at 5-8 queues in any mix the cost was -3 to +2.5 %
// (tools/svc_interference.py with HIP's queue log, profiles/r6/queues/).  So
// the library's own footprint stays within 8: the normal class (shared with
// every other stream of the process), the low-priority H2D copy queue of the
// host paths, and at most 8 - normal - low service queues (3 by default).
constexpr int kProcessHwQueues = 8;
int svc_queue_cap() {
  static const int cap = [] {
    int q = 4;  // HIP's default GPU_MAX_HW_QUEUES
    if (const char* env = std::getenv("GPU_MAX_HW_QUEUES"))
      if (std::atoi(env) > 0) q = std::atoi(env);
    q = std::min(q, 32);
    return std::max(1, std::min(q, kProcessHwQueues - q - 1));
  }();
  return cap;
}

// A stream of the pool for c's service, or null when every pool stream of the
// device is leased.  Called under the context's DeviceGuard.
hipStream_t svc_lease(ugo_fec* c) {
  SvcStreamPool& p = svc_pool();
  std::lock_guard<std::mutex> lk(p.mu);
  std::vector<hipStream_t>& idle = p.idle[c->device];
  if (!idle.empty()) {
    hipStream_t s = idle.back();
    idle.pop_back();
    return s;
  }
  int& made = p.created[c->device];
  if (made >= svc_queue_cap()) return nullptr;
  hipStream_t s = nullptr;
  if (create_service_stream(c->device, &s) != hipSuccess) return nullptr;
  ++made;
  return s;
}

// Back to the pool: only once no block of c's can still be resident on it.
void svc_release(ugo_fec* c) {
  if (!c->svc_stream) return;
  SvcStreamPool& p = svc_pool();
  std::lock_guard<std::mutex> lk(p.mu);
  p.idle[c->device].push_back(c->svc_stream);
  c->svc_stream = nullptr;
}

// A stream whose block faulted: destroyed, not pooled; its slot is counted
// free so the next lease makes a fresh stream.
void svc_discard(ugo_fec* c) {
  if (!c->svc_stream) return;
  (void)hipGetLastError();
  (void)hipStreamDestroy(c->svc_stream);
  c->svc_stream = nullptr;
  SvcStreamPool& p = svc_pool();
  std::lock_guard<std::mutex> lk(p.mu);
  int& made = p.created[c->device];
  if (made > 0) --made;
}

// Writes one request (layout: SvcBox::line): every field, then the pieces'
// tags, then seq; returns seq.
uint32_t svc_post(ugo_fec* c, uint32_t op, const uint8_t* mapped, size_t groups, size_t S, size_t pitch,
                  unsigned flags, const uint64_t* present) {
  ugo::kern::SvcBox* b = c->svc_box;
  uint32_t* l = b->line;
  const uint64_t sh = reinterpret_cast<uint64_t>(mapped);
  const uint64_t m0 = present && groups > 0 ? present[0] : 0, m1 = present && groups > 1 ? present[1] : 0;
  if (present && groups > 2) std::memcpy(b->present + 2, present + 2, (groups - 2) * sizeof(uint64_t));
  l[1] = op;
  l[2] = static_cast<uint32_t>(groups);
  l[3] = static_cast<uint32_t>(S);
  l[5] = static_cast<uint32_t>(sh);
  l[6] = static_cast<uint32_t>(sh >> 32);
  l[7] = (flags & UGO_FEC_RECONSTRUCT_DATA_ONLY) ? 1u : 0u;
  l[9] = static_cast<uint32_t>(pitch);
  l[10] = static_cast<uint32_t>(uint64_t(pitch) >> 32);
  l[11] = static_cast<uint32_t>(m0);
  l[13] = static_cast<uint32_t>(m0 >> 32);
  l[14] = static_cast<uint32_t>(m1);
  l[15] = static_cast<uint32_t>(m1 >> 32);
  const uint32_t sq = ++c->svc_seq;
  svc_st(l[4], sq);
  svc_st(l[8], sq);
  svc_st(l[12], sq);
  svc_st(l[0], sq);  // release: everything above is visible first
  return sq;
}

// A HIP status of the service stream that means the block died (any error:
// a fault, an illegal address, a launch timeout -- not "still running").
bool svc_faulted(ugo_fec* c) {
  const hipError_t q = hipStreamQuery(c->svc_stream);
  if (q == hipSuccess || q == hipErrorNotReady) return false;
  return true;
}

// Makes sure no service block is left: posts a stop if one is alive, then
// waits up to the grace period for it to clear `alive` and for its stream to
// drain.  OK: gone (or dead), nothing it could still write.  Otherwise the
// context is poisoned.
int svc_retire(ugo_fec* c) {
  c->svc_on = false;
  if (!c->svc_box || !c->svc_stream) return UGO_FEC_OK;
  ugo::kern::SvcBox* b = c->svc_box;
  if (svc_ld(b->alive)) (void)svc_post(c, ugo::kern::kSvcStop, nullptr, 0, 0, 0, 0, nullptr);
  const auto t0 = std::chrono::steady_clock::now();
  const auto grace = std::chrono::milliseconds(c->svc_grace_ms);
  for (uint32_t spin = 0;; ++spin) {
    if ((spin & 255u) == 0) {
      const hipError_t q = hipStreamQuery(c->svc_stream);
      // drained (alive is 0 or the block never ran): nothing of c's is left on
      // the stream, another context may lease it.  Faulted (the block is dead):
      // nothing of c's runs either, but the stream may carry the fault's sticky
      // state, so it is dropped and its pool slot freed for a fresh stream
      // 
      if (q == hipSuccess) {
        svc_release(c);
        return UGO_FEC_OK;
      }
      if (q != hipErrorNotReady) {
        svc_discard(c);
        return UGO_FEC_OK;
      }
      if (std::chrono::steady_clock::now() - t0 > grace) break;
    }
    svc_relax();
  }
  c->poisoned = true;  // the stream stays leased: the block may still be on it
  return UGO_FEC_ERR_HIP;
}

// One request: op on `groups` (<= kSvcMaxGroups) groups of the pinned
// group-major batch at `mapped` (device view).  Statuses as the launch path.
int svc_call(ugo_fec* c, uint32_t op, uint8_t* mapped, size_t groups, size_t S, size_t pitch, unsigned flags,
             const uint64_t* present, int8_t* status) {
  ugo::kern::SvcBox* b = c->svc_box;
  if (!svc_ld(b->alive) && svc_launch(c, c->svc_seq) != UGO_FEC_OK) return UGO_FEC_ERR_HIP;
  const uint32_t sq = svc_post(c, op, mapped, groups, S, pitch, flags, present);
  const auto t0 = std::chrono::steady_clock::now();
  const auto limit = std::chrono::milliseconds(c->svc_timeout_ms);
  for (uint32_t spin = 0; svc_ld(b->done) != sq; ++spin) {
    if (!svc_ld(b->alive)) {  // it left before it saw this request
      if (svc_ld(b->done) == sq) break;
      if (svc_launch(c, sq - 1) != UGO_FEC_OK) {
        (void)svc_retire(c);
        return UGO_FEC_ERR_HIP;
      }
    }
    if ((spin & 1023u) == 0 && (svc_faulted(c) || std::chrono::steady_clock::now() - t0 > limit)) {
      // a faulted or silent block: it must be gone before this call returns (it
      // may still be serving sq into the caller's batch); later calls take the
      // launch path, or fail if it never leaves (poisoned)
      (void)svc_retire(c);
      return UGO_FEC_ERR_HIP;
    }
    svc_relax();
  }
  if (op != ugo::kern::kSvcReconstruct) return UGO_FEC_OK;
  int first = UGO_FEC_OK;
  for (size_t g = 0; g < groups; ++g) {
    const int8_t v = b->status[g];
    if (status) status[g] = v;
    if (v && !first) first = v;
  }
  return first;
}

int svc_stop(ugo_fec* c) {
  if (!c->svc_box) return UGO_FEC_OK;
  return svc_retire(c);
}

// Host path: chunks of stage_groups groups round-robin over kStreams streams:
// H2D(chunk) -> kernel -> D2H(chunk) on one stream, chunks on different
// streams overlap (copy engines in both directions + compute).
int host_path(ugo_fec* c, uint8_t* shards, const uint64_t* present, size_t groups, size_t S,
              size_t pitch, bool recon, unsigned flags, int8_t* status) {
  int st = UGO_FEC_OK;
  const size_t gbytes = size_t(c->n) * pitch;
  std::vector<int8_t> tmp_status;
  if (recon && !status) {
    tmp_status.resize(groups);
    status = tmp_status.data();
  }
  // Reconstruct of a pinned batch: zero-copy.  The kernels run on the batch's
  // device mapping, reading the d survivor rows of each group over PCIe and
  // writing the erased rows back in place -- d rows in per group instead of the
  // staged path's d + p (tools/zerocopy_probe.py: (10,3) 13.3 vs 23.8 ms,
  // (32,8) 40.6 vs 62.6 ms).  Only the masks and statuses are staged.  A large
  // encode stays staged: its DMA copies beat zero-copy reads (16.2 vs 18.5 ms).
  uint8_t* mapped = nullptr;
  {
    hipPointerAttribute_t at{};
    if (hipPointerGetAttributes(&at, shards) == hipSuccess && at.type == hipMemoryTypeHost && at.devicePointer) {
      mapped = static_cast<uint8_t*>(at.devicePointer);
      if (at.hostPointer && at.hostPointer != at.devicePointer)
        mapped += shards - static_cast<uint8_t*>(at.hostPointer);  // interior pointer
      else
        mapped = shards;
    } else {
      (void)hipGetLastError();  // pageable: clear the sticky lookup error
    }
  }
  if (svc_eligible(c, mapped, groups, pitch, recon))
    return svc_call(c, recon ? ugo::kern::kSvcReconstruct : ugo::kern::kSvcEncode, mapped, groups, S, pitch, flags,
                    recon ? present : nullptr, status);
  if (recon && mapped) return host_reconstruct_mapped(c, mapped, present, groups, S, pitch, flags, status);
  // Encode of a small pinned batch (the per-group calls of the drop-in
  // reedsolomon::Encoder, calcECC): zero-copy too -- one launch reading the data
  // rows and writing the parity rows through the mapping, one synchronize --
  // instead of the three-copy pipeline, whose DMA only wins on large batches.
  if (!recon && mapped && groups * gbytes <= kZeroCopyEncodeBytes) {
    if (!c->streams[0] && hipStreamCreateWithFlags(&c->streams[0], hipStreamNonBlocking) != hipSuccess)
      return UGO_FEC_ERR_HIP;
    hipStream_t s = c->streams[0];
    st = encode_dev(c, mapped, groups, S, interleaved(c, pitch), s);
    if (st) return st;
    return hip_status(hipStreamSynchronize(s));
  }
  // staged (pageable batches, large pinned encodes): the stage buffers and streams only now -- a
  // context served by the service or zero-copy (one per connection) never holds 3 x 64 MiB of stage
  st = ensure_stage(c, pitch);
  if (st) return st;
  const size_t per = c->stage_groups;
  size_t chunk = 0;
  for (size_t g0 = 0; g0 < groups; g0 += per, ++chunk) {
    const int si = static_cast<int>(chunk % kStreams);
    hipStream_t s = c->streams[si];
    const size_t gn = std::min(per, groups - g0);
    uint8_t* host = shards + g0 * gbytes;
    uint8_t* dev = c->d_stage[si];
    hipError_t e;
    if (!recon) {
      // data rows in, parity rows out
      e = hipMemcpy2DAsync(dev, gbytes, host, gbytes, size_t(c->d) * pitch, gn, hipMemcpyHostToDevice, s);
      if (e != hipSuccess) return UGO_FEC_ERR_HIP;
      st = encode_dev(c, dev, gn, S, interleaved(c, pitch), s);
      if (st) return st;
      // parity rows out, bytes [0, S) only: padding bytes of the caller's rows are never written
      hipMemcpy3DParms cp{};
      cp.srcPtr = make_hipPitchedPtr(dev, pitch, pitch, c->n);
      cp.srcPos = make_hipPos(0, c->d, 0);
      cp.dstPtr = make_hipPitchedPtr(host, pitch, pitch, c->n);
      cp.dstPos = make_hipPos(0, c->d, 0);
      cp.extent = make_hipExtent(S, c->p, gn);
      cp.kind = hipMemcpyDeviceToHost;
      e = hipMemcpy3DAsync(&cp, s);
      if (e != hipSuccess) return UGO_FEC_ERR_HIP;
    } else {
      const size_t W = mask_words(c);
      e = hipMemcpyAsync(dev, host, gn * gbytes, hipMemcpyHostToDevice, s);
      if (e == hipSuccess)
        e = hipMemcpyAsync(c->d_mask[si], present + g0 * W, gn * W * sizeof(uint64_t), hipMemcpyHostToDevice, s);
      if (e != hipSuccess) return UGO_FEC_ERR_HIP;
      st = reconstruct_dev(c, dev, c->d_mask[si], gn, S, interleaved(c, pitch), flags, c->d_status[si], s, {},
                           present + g0 * W);
      if (st) return st;
      // all rows back: present rows and padding come back byte-identical (they
      // were copied in above and the kernels write only erased rows' [0, S))
      e = hipMemcpyAsync(host, dev, gn * gbytes, hipMemcpyDeviceToHost, s);
      if (e == hipSuccess) e = hipMemcpyAsync(status + g0, c->d_status[si], gn, hipMemcpyDeviceToHost, s);
      if (e != hipSuccess) return UGO_FEC_ERR_HIP;
    }
  }
  for (int i = 0; i < kStreams; ++i)
    if (hipStreamSynchronize(c->streams[i]) != hipSuccess) return UGO_FEC_ERR_HIP;
  if (recon)
    for (size_t g = 0; g < groups; ++g)
      if (status[g]) return status[g];
  return UGO_FEC_OK;
}

// Bytes a frame row is written to: round_up(S + 6, 16), or -- when the row
// slots are 64-B aligned and span it -- round_up(S + 6, 64): a row then ends on
// a whole 64-B line instead of leaving its last line partially written (which
// the neighbouring row's writer completes at another time).
#ifndef UGO_RX_FRAME_FILL64
#define UGO_RX_FRAME_FILL64 1
#endif
size_t rx_frame_fill(const uint8_t* shards, size_t S, size_t rstride, size_t gstride, size_t rows, size_t groups) {
  const size_t w16 = round_up(S + 6, 16), w64 = round_up(S + 6, 64);
  if (!UGO_RX_FRAME_FILL64 || reinterpret_cast<uintptr_t>(shards) % 64 || rstride % 64 || gstride % 64) return w16;
  return layout_disjoint(w64, rstride, rows, gstride, groups) ? w64 : w16;
}

// Stream-ordered scratch of one rx_assemble call: presence snapshot [groups] u64 | claim words
// [groups][n] u32 | dup flag.
size_t rx_scratch_bytes(const ugo_fec* c, size_t groups) {
  return groups * sizeof(uint64_t) + (groups * size_t(c->n) + 16) * sizeof(uint32_t);
}

// rx_assemble on device views (arguments checked by the caller).
int rx_assemble_dev(ugo_fec* c, const uint8_t* wire, size_t slot_stride, const uint16_t* lens, size_t npk,
                    const uint8_t* pad, uint64_t first_group, size_t groups, uint8_t* shards, size_t S,
                    size_t row_stride, size_t group_stride, uint64_t* present, uint32_t* stats, hipStream_t s,
                    bool frame = false, void* call_scratch = nullptr) {
  ugo::kern::RxArgs a{};
  a.frame = frame ? 1u : 0u;
  a.fill = static_cast<uint32_t>(rx_frame_fill(shards, S, row_stride, group_stride, size_t(c->n), groups));
  a.wire = wire;
  a.lens = lens;
  a.pad = pad;
  a.shards = shards;
  a.present = present;
  a.stats = stats;
  a.npk = npk;
  a.slot = slot_stride;
  a.first_group = first_group;
  a.groups = groups;
  a.rstride = row_stride;
  a.gstride = group_stride;
  a.S = static_cast<uint32_t>(S);
  a.n = static_cast<uint32_t>(c->n);
  // First arrival in ring order wins (ugo/fec.go:123-129), optimistically
  // (rx_kernels.hip): place everything, flag a (group, row) taken twice, and
  // only then -- gated on the flag, on the device -- claim and re-place.
  // scratch: presence snapshot [groups] u64 | claim words [groups][n] u32 | dup flag
  const uint64_t words = groups * uint64_t(c->n);
  // call_scratch: the caller's (rx_recover_host: one block for all its chunk calls, which run in order on s),
  // rx_scratch_bytes(c, groups) of it
  void* scratch = call_scratch;
  int st = call_scratch ? UGO_FEC_OK : scratch_alloc(c, rx_scratch_bytes(c, groups), s, &scratch);
  if (st) return st;
  uint64_t* prev = static_cast<uint64_t*>(scratch);
  uint32_t* win = reinterpret_cast<uint32_t*>(prev + groups);
  uint32_t* dup = win + words;
  // call entry, one launch: dup = 0, the presence snapshot -- a (group, row)
  // an earlier call placed keeps that call's copy (ugo/fec.go:123-129 keeps the
  // first) -- the claim words, and whether any presence bit was set at all (if
  // none was, the place pass skips its per-packet snapshot lookups)
  const unsigned long long call = ++c->rx_calls;
  st = hip_status(ugo::kern::launch_rx_begin(present, prev, groups, dup, win, words, c->d_rxseen, call, s));
  a.dup = dup;
  a.prev = prev;
  a.seen = c->d_rxseen;
  a.call = call;
  ugo::kern::RxArgs f = a;  // the gated claim and re-place of the first copies
  f.win = win;
  f.gate = dup;
  f.dup = nullptr;
  f.stats = nullptr;
  f.fixup = 1;
  if (!st) st = hip_status(ugo::kern::launch_rx_scatter(a, s));
  if (!st) st = hip_status(ugo::kern::launch_rx_claim(f, s));
  if (!st) st = hip_status(ugo::kern::launch_rx_scatter(f, s));
  const int fr = call_scratch ? UGO_FEC_OK : scratch_free(c, scratch, s);
  return st ? st : fr;
}


// ugo_fec_lossy_groups on device views: one launch (k_lossy_list1), or the
// two-launch form (k_lossy_count -> k_lossy_write) in A/B builds.
#ifndef UGO_LOSSY_ONE_LAUNCH
#define UGO_LOSSY_ONE_LAUNCH 1
#endif
constexpr bool kLossyOneLaunch = UGO_LOSSY_ONE_LAUNCH != 0;
int lossy_list_dev(ugo_fec* c, const uint64_t* present, size_t groups, unsigned flags, uint32_t* list,
                   uint32_t* count, hipStream_t s, uint32_t* rowoff = nullptr, uint32_t* rows = nullptr) {
  if (groups == 0) {
    if (rows && hipMemsetAsync(rows, 0, sizeof(uint32_t), s) != hipSuccess) return UGO_FEC_ERR_HIP;
    return hip_status(hipMemsetAsync(count, 0, sizeof(uint32_t), s));
  }
  const uint64_t nmask = c->n >= 64 ? ~0ull : ((1ull << c->n) - 1);
  const uint64_t dmask =
      (flags & UGO_FEC_RECONSTRUCT_DATA_ONLY) && c->d < 64 ? ((1ull << c->d) - 1) : ~0ull;  // d = 64: p = 0
  const size_t blocks = (groups + ugo::kern::kLossyPerBlock - 1) / ugo::kern::kLossyPerBlock;
  if (kLossyOneLaunch) {
    // the stream's count words (made, or grown, on first use; zeroed once, on the call's own stream so the
    // zeroing is ordered before the kernel -- hipMemset is asynchronous to a non-blocking stream -- and
    // epoch 0 is never used)
    ugo_fec::LossyWords* lw = nullptr;
    for (auto& e : c->lossy_words)
      if (e.s == s) lw = &e;
    if (!lw || lw->tiles < blocks || lw->epoch == 0xffffffffu) {
      if (lw && hipStreamSynchronize(s) != hipSuccess) return UGO_FEC_ERR_HIP;
      const size_t tiles = std::max<size_t>(blocks, lw ? 2 * lw->tiles : 64);
      uint64_t* w = nullptr;
      if (hipMalloc(&w, tiles * sizeof(uint64_t)) != hipSuccess) return UGO_FEC_ERR_HIP;
      if (hipMemsetAsync(w, 0, tiles * sizeof(uint64_t), s) != hipSuccess) {
        (void)hipFree(w);
        return UGO_FEC_ERR_HIP;
      }
      if (lw) {
        (void)hipFree(lw->words);
        *lw = ugo_fec::LossyWords{s, w, tiles, 0};
      } else {
        c->lossy_words.push_back(ugo_fec::LossyWords{s, w, tiles, 0});
        lw = &c->lossy_words.back();
      }
    }
    const uint32_t epoch = ++lw->epoch;
    return hip_status(ugo::kern::launch_lossy_list1(present, groups, nmask, dmask, static_cast<uint32_t>(c->d), list,
                                                    count, rowoff, rows, lw->words, epoch, s));
  }
  void* work = nullptr;
  int st = scratch_alloc(c, 2 * blocks * sizeof(uint32_t), s, &work);
  if (st) return st;
  st = hip_status(ugo::kern::launch_lossy_list(present, groups, nmask, dmask, static_cast<uint32_t>(c->d), list,
                                               count, rowoff, rows, static_cast<uint32_t*>(work), s));
  const int fr = scratch_free(c, work, s);
  return st ? st : fr;
}

// ugo_fec_reconstruct_list on device views (arguments checked by the caller).
int reconstruct_list_dev(ugo_fec* c, const uint8_t* shards, const uint64_t* present, const uint32_t* list,
                         const uint32_t* count, size_t max_entries, size_t S, const Layout& L, uint8_t* out,
                         size_t out_row_stride, size_t out_entry_stride, unsigned flags, int8_t* status,
                         hipStream_t s, const uint32_t* rowoff = nullptr, uint32_t* rowid = nullptr,
                         uint32_t max_rows = 0xffffffffu) {
  ugo::kern::Batch a = base_batch(c, const_cast<uint8_t*>(shards), S, L);
  a.rowoff = rowoff;  // row-compact outputs (rx_recover_host, ugo_fec_recover_data)
  a.rowid = rowid;
  a.max_rows = max_rows;
  a.n = static_cast<uint32_t>(c->n);
  a.out = out;
  a.ogstride = out_entry_stride;
  a.orstride = out_row_stride;
  a.present = present;
  a.status = status;
  a.data_only = (flags & UGO_FEC_RECONSTRUCT_DATA_ONLY) ? 1u : 0u;
  a.chunks = static_cast<uint32_t>((S + 15) / 16);
  a.desc = c->d_table;
  a.list = list;
  a.count = count;
  const size_t per = slice_groups(a.chunks, true);
  for (size_t g0 = 0; g0 < max_entries; g0 += per) {
    const size_t gn = std::min(per, max_entries - g0);
    a.g0 = g0;
    a.items = static_cast<uint32_t>(gn * a.chunks);
    if (ugo::kern::launch_apply_list(ugo::kern::apply_dmax(c->d), a, s) != hipSuccess) return UGO_FEC_ERR_HIP;
  }
  return UGO_FEC_OK;
}


}  // namespace

extern "C" {

int ugo_fec_abi_version(void) { return UGO_FEC_ABI_VERSION; }

const char* ugo_fec_strerror(int s) {
  switch (s) {
    case UGO_FEC_OK: return "ok";
    case UGO_FEC_ERR_INV_SHARD_NUM:
      return "cannot create Encoder with less than one data shard or less than zero parity shards";
    case UGO_FEC_ERR_MAX_SHARD_NUM: return "cannot create Encoder with more than 256 data+parity shards";
    case UGO_FEC_ERR_TOO_FEW_SHARDS: return "too few shards given";
    case UGO_FEC_ERR_SHARD_NO_DATA: return "no shard data";
    case UGO_FEC_ERR_SHARD_SIZE: return "shard sizes do not match";
    case UGO_FEC_ERR_INVALID_ARG: return "invalid argument";
    case UGO_FEC_ERR_SINGULAR: return "matrix is singular";
    case UGO_FEC_ERR_HIP: return "HIP runtime error";
    case UGO_FEC_ERR_NO_DEVICE: return "no usable gfx950 device";
    default: return "unknown status";
  }
}

int ugo_fec_check_shards(int n, const size_t* lens, int nil_ok, size_t* shard_size) {
  if (n <= 0 || !lens) return UGO_FEC_ERR_INVALID_ARG;
  size_t size = 0;
  for (int i = 0; i < n; ++i)
    if (lens[i]) {
      size = lens[i];
      break;
    }
  if (shard_size) *shard_size = size;
  if (size == 0) return UGO_FEC_ERR_SHARD_NO_DATA;
  for (int i = 0; i < n; ++i)
    if (lens[i] != size && (lens[i] != 0 || !nil_ok)) return UGO_FEC_ERR_SHARD_SIZE;
  return UGO_FEC_OK;
}

int ugo_fec_create(int device, int data_shards, int parity_shards, ugo_fec** out) {
  if (!out) return UGO_FEC_ERR_INVALID_ARG;
  *out = nullptr;
  if (data_shards <= 0 || parity_shards < 0) return UGO_FEC_ERR_INV_SHARD_NUM;
  if (data_shards + parity_shards > 256) return UGO_FEC_ERR_MAX_SHARD_NUM;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || device < 0 || device >= count) return UGO_FEC_ERR_NO_DEVICE;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) return UGO_FEC_ERR_NO_DEVICE;
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return UGO_FEC_ERR_NO_DEVICE;
  DeviceGuard guard(device);
  if (!guard.ok) return UGO_FEC_ERR_NO_DEVICE;

  ugo_fec* c = new (std::nothrow) ugo_fec();
  if (!c) return UGO_FEC_ERR_INVALID_ARG;
  c->device = device;
  c->d = data_shards;
  c->p = parity_shards;
  c->n = data_shards + parity_shards;
  if (const char* env = std::getenv("UGO_FEC_TABLE_MAX_SHARDS")) c->table_max = std::atoi(env);
  const int d = c->d, p = c->p, n = c->n;
  c->M.resize(size_t(n) * d);
  std::vector<uint8_t> scratch(size_t(n) * d + 3 * size_t(d) * d);
  if (!ugo::gf::build_matrix(d, p, c->M.data(), scratch.data())) {
    delete c;
    return UGO_FEC_ERR_SINGULAR;
  }
  const int dmax = ugo::kern::apply_dmax(d);
  c->dpad = static_cast<uint32_t>(round_up(std::max(d, dmax), 4));
  c->epad = static_cast<uint32_t>(round_up(std::max(p, 1), 4));
  c->desc_stride = static_cast<uint32_t>(round_up(4 + c->dpad + c->epad + size_t(p) * c->dpad, 16));

  int st = UGO_FEC_OK;
  auto fail = [&](int code) {
    free_ctx(c);
    return code;
  };
  if (hipMalloc(&c->d_M, c->M.size()) != hipSuccess) return fail(UGO_FEC_ERR_HIP);
  if (hipMemcpy(c->d_M, c->M.data(), c->M.size(), hipMemcpyHostToDevice) != hipSuccess) return fail(UGO_FEC_ERR_HIP);
  {
    std::vector<uint8_t> gf(1024 + 256 * 32, 0);  // exp | log | pad | perm tables
    std::memcpy(gf.data(), ugo::gf::kTables.exp, 512);
    std::memcpy(gf.data() + 512, ugo::gf::kTables.log, 256);
    ugo::gf::perm_tables(gf.data() + 1024);
    if (hipMalloc(&c->d_gf, gf.size()) != hipSuccess) return fail(UGO_FEC_ERR_HIP);
    if (hipMemcpy(c->d_gf, gf.data(), gf.size(), hipMemcpyHostToDevice) != hipSuccess) return fail(UGO_FEC_ERR_HIP);
  }
  {
    // MODE 0 encode descriptor: inputs = data rows, outputs = parity rows
    std::vector<uint8_t> ed(c->desc_stride + 64, 0);
    ed[0] = static_cast<uint8_t>(p);
    ed[1] = 0;
    for (int i = 0; i < d; ++i) ed[4 + i] = static_cast<uint8_t>(i);
    for (int i = 0; i < p; ++i) ed[4 + c->dpad + i] = static_cast<uint8_t>(d + i);
    for (int i = 0; i < p; ++i)
      for (int k = 0; k < d; ++k) ed[4 + c->dpad + c->epad + size_t(i) * c->dpad + k] = c->M[size_t(d + i) * d + k];
    if (hipMalloc(&c->d_encdesc, ed.size()) != hipSuccess) return fail(UGO_FEC_ERR_HIP);
    if (hipMemcpy(c->d_encdesc, ed.data(), ed.size(), hipMemcpyHostToDevice) != hipSuccess) return fail(UGO_FEC_ERR_HIP);
    if (hipMalloc(&c->d_rxseen, sizeof(unsigned long long)) != hipSuccess ||
        hipMemset(c->d_rxseen, 0, sizeof(unsigned long long)) != hipSuccess)
      return fail(UGO_FEC_ERR_HIP);
  }
  if (n <= c->table_max && n <= 20) {
    const size_t entries = size_t(1) << n;
    std::vector<uint8_t> tab(entries * c->desc_stride + 64, 0);
    for (size_t m = 0; m < entries; ++m) {
      st = build_desc(c, m, &tab[m * c->desc_stride]);
      if (st) return fail(st);
    }
    if (hipMalloc(&c->d_table, tab.size()) != hipSuccess) return fail(UGO_FEC_ERR_HIP);
    if (hipMemcpy(c->d_table, tab.data(), tab.size(), hipMemcpyHostToDevice) != hipSuccess) return fail(UGO_FEC_ERR_HIP);
  }
  *out = c;
  return UGO_FEC_OK;
}

void ugo_fec_destroy(ugo_fec* c) { free_ctx(c); }

int ugo_fec_geometry(const ugo_fec* c, int* d, int* p, int* device) {
  if (!c) return UGO_FEC_ERR_INVALID_ARG;
  if (d) *d = c->d;
  if (p) *p = c->p;
  if (device) *device = c->device;
  return UGO_FEC_OK;
}

int ugo_fec_matrix(const ugo_fec* c, uint8_t* out) {
  if (!c || !out) return UGO_FEC_ERR_INVALID_ARG;
  std::memcpy(out, c->M.data(), c->M.size());
  return UGO_FEC_OK;
}

int ugo_fec_encode_strided(ugo_fec* c, uint8_t* shards, size_t groups, size_t S, size_t row_stride,
                           size_t group_stride, void* stream) {
  const Layout L{row_stride, group_stride};
  int st = check_batch(c, shards, groups, S, L);
  if (st) return st;
  DeviceGuard g(c->device);
  if (!g.ok) return UGO_FEC_ERR_NO_DEVICE;
  if (groups == 0) return UGO_FEC_OK;  // nothing is touched (an empty tensor's pointer may be anything)
  if (!device_view(shards)) return UGO_FEC_ERR_INVALID_ARG;
  TimerScope ts(c);
  return encode_dev(c, shards, groups, S, L, static_cast<hipStream_t>(stream));
}

int ugo_fec_encode(ugo_fec* c, uint8_t* shards, size_t groups, size_t S, size_t pitch, void* stream) {
  if (!c) return UGO_FEC_ERR_INVALID_ARG;
  if (c->poisoned) return UGO_FEC_ERR_HIP;  // a service block that never left (svc_retire)
  if (pitch < S) return S == 0 ? UGO_FEC_ERR_SHARD_NO_DATA : UGO_FEC_ERR_INVALID_ARG;
  return ugo_fec_encode_strided(c, shards, groups, S, pitch, size_t(c->n) * pitch, stream);
}

int ugo_fec_reconstruct_strided(ugo_fec* c, uint8_t* shards, const uint64_t* present, size_t groups, size_t S,
                                size_t row_stride, size_t group_stride, unsigned flags, int8_t* status,
                                void* stream) {
  const Layout L{row_stride, group_stride};
  int st = check_batch(c, shards, groups, S, L);
  if (st) return st;
  DeviceGuard g(c->device);
  if (!g.ok) return UGO_FEC_ERR_NO_DEVICE;
  if (groups == 0) return UGO_FEC_OK;
  if (!device_view(shards) || !device_view(present) || !device_view(status)) return UGO_FEC_ERR_INVALID_ARG;
  TimerScope ts(c);
  return reconstruct_dev(c, shards, present, groups, S, L, flags, status, static_cast<hipStream_t>(stream));
}

int ugo_fec_reconstruct_into(ugo_fec* c, const uint8_t* shards, const uint64_t* present, size_t groups, size_t S,
                             size_t row_stride, size_t group_stride, uint8_t* out, size_t out_row_stride,
                             size_t out_group_stride, unsigned flags, int8_t* status, void* stream) {
  const Layout L{row_stride, group_stride};
  int st = check_batch(c, shards, groups, S, L);
  if (st) return st;
  if (groups == 0) return UGO_FEC_OK;
  // p output slots of S bytes per group: no two slots may overlap (the smaller
  // stride must clear S, the larger one a whole run of the smaller), and the
  // output may not overlap the batch it reads (other lanes would read rows
  // being overwritten)
  if (!out || !layout_disjoint(S, out_row_stride, size_t(c->p), out_group_stride, groups)) return UGO_FEC_ERR_INVALID_ARG;
  {
    const size_t in_ext = extent(S, row_stride, size_t(c->n), group_stride, groups);
    const size_t out_ext = extent(S, out_row_stride, size_t(c->p), out_group_stride, groups);
    const uintptr_t i0 = reinterpret_cast<uintptr_t>(shards), o0 = reinterpret_cast<uintptr_t>(out);
    if (o0 < i0 + in_ext && i0 < o0 + out_ext) return UGO_FEC_ERR_INVALID_ARG;
  }
  DeviceGuard g(c->device);
  if (!g.ok) return UGO_FEC_ERR_NO_DEVICE;
  if (!device_view(shards) || !device_view(present) || !device_view(status) || !device_view(out))
    return UGO_FEC_ERR_INVALID_ARG;
  TimerScope ts(c);
  OutBatch O;
  O.base = out;
  O.L = Layout{out_row_stride, out_group_stride};
  return reconstruct_dev(c, const_cast<uint8_t*>(shards), present, groups, S, L, flags, status,
                         static_cast<hipStream_t>(stream), O);
}

int ugo_fec_lossy_groups(ugo_fec* c, const uint64_t* present, size_t groups, unsigned flags, uint32_t* list,
                         uint32_t* count, void* stream) {
  if (!c) return UGO_FEC_ERR_INVALID_ARG;
  if (c->poisoned) return UGO_FEC_ERR_HIP;  // a service block that never left (svc_retire)
  if (!present || !list || !count || c->n > 64 || groups >= 0xffffffffull) return UGO_FEC_ERR_INVALID_ARG;
  DeviceGuard g(c->device);
  if (!g.ok) return UGO_FEC_ERR_NO_DEVICE;
  if (!device_view(present) || !device_view(list) || !device_view(count)) return UGO_FEC_ERR_INVALID_ARG;
  TimerScope ts(c);
  return lossy_list_dev(c, present, groups, flags, list, count, static_cast<hipStream_t>(stream));
}

int ugo_fec_reconstruct_list(ugo_fec* c, const uint8_t* shards, const uint64_t* present, size_t groups,
                             const uint32_t* list, const uint32_t* count, size_t max_entries, size_t S,
                             size_t row_stride, size_t group_stride, uint8_t* out, size_t out_row_stride,
                             size_t out_entry_stride, unsigned flags, int8_t* status, void* stream) {
  const Layout L{row_stride, group_stride};
  int st = check_batch(c, shards, groups, S, L);
  if (st) return st;
  if (groups == 0 || max_entries == 0) return UGO_FEC_OK;
  if (!present || !list || !count || c->n > 16 || !c->d_table || max_entries > groups)
    return UGO_FEC_ERR_INVALID_ARG;
  if (!fast_layout(c, shards, L, S)) return UGO_FEC_ERR_INVALID_ARG;
  const size_t oslots = (flags & UGO_FEC_RECONSTRUCT_DATA_ONLY) ? size_t(std::min(c->d, c->p)) : size_t(c->p);
  if (out) {
    if (reinterpret_cast<uintptr_t>(out) % 16 || out_row_stride % 16 || out_entry_stride % 16 ||
        !layout_disjoint(S, out_row_stride, oslots, out_entry_stride, max_entries))
      return UGO_FEC_ERR_INVALID_ARG;
    const size_t in_ext = extent(S, row_stride, size_t(c->n), group_stride, groups);
    const size_t out_ext = extent(S, out_row_stride, oslots, out_entry_stride, max_entries);
    const uintptr_t i0 = reinterpret_cast<uintptr_t>(shards), o0 = reinterpret_cast<uintptr_t>(out);
    if (o0 < i0 + in_ext && i0 < o0 + out_ext) return UGO_FEC_ERR_INVALID_ARG;
  }
  DeviceGuard g(c->device);
  if (!g.ok) return UGO_FEC_ERR_NO_DEVICE;
  if (!device_view(shards) || !device_view(present) || !device_view(list) || !device_view(count) ||
      !device_view(status) || !device_view(out))
    return UGO_FEC_ERR_INVALID_ARG;
  TimerScope ts(c);
  return reconstruct_list_dev(c, shards, present, list, count, max_entries, S, L, out, out_row_stride,
                              out_entry_stride, flags, status, static_cast<hipStream_t>(stream));
}

int ugo_fec_recover_data(ugo_fec* c, const uint8_t* shards, const uint64_t* present, size_t groups, size_t S,
                         size_t row_stride, size_t group_stride, uint8_t* out, size_t out_row_stride, size_t max_rows,
                         uint32_t* index, uint32_t* count, void* stream) {
  const Layout L{row_stride, group_stride};
  int st = check_batch(c, shards, groups, S, L);
  if (st) return st;
  if (!present || !count || c->n > 16 || !c->d_table || groups * size_t(c->n) >= 0xffffffffull ||
      max_rows > 0xffffffffull || (max_rows && (!out || !index)))
    return UGO_FEC_ERR_INVALID_ARG;
  if (!fast_layout(c, shards, L, S)) return UGO_FEC_ERR_INVALID_ARG;
  if (max_rows) {
    if (reinterpret_cast<uintptr_t>(out) % 16 || out_row_stride % 16 || out_row_stride < round_up(S, 16))
      return UGO_FEC_ERR_INVALID_ARG;
    const size_t in_ext = extent(S, row_stride, size_t(c->n), group_stride, groups);
    const size_t out_ext = (max_rows - 1) * out_row_stride + S;
    const uintptr_t i0 = reinterpret_cast<uintptr_t>(shards), o0 = reinterpret_cast<uintptr_t>(out);
    if (o0 < i0 + in_ext && i0 < o0 + out_ext) return UGO_FEC_ERR_INVALID_ARG;
  }
  DeviceGuard g(c->device);
  if (!g.ok) return UGO_FEC_ERR_NO_DEVICE;
  if (!device_view(shards) || !device_view(present) || !device_view(out) || !device_view(index) ||
      !device_view(count))
    return UGO_FEC_ERR_INVALID_ARG;
  TimerScope ts(c);
  const hipStream_t s = static_cast<hipStream_t>(stream);
  if (groups == 0) return hip_status(hipMemsetAsync(count, 0, sizeof(uint32_t), s));
  // scratch: the lossy-group list | each entry's first output row | the entry count
  void* scratch = nullptr;
  st = scratch_alloc(c, groups * 8 + 16, s, &scratch);
  if (st) return st;
  uint32_t* list = static_cast<uint32_t*>(scratch);
  uint32_t* rowoff = list + groups;
  uint32_t* entries = rowoff + groups;
  st = lossy_list_dev(c, present, groups, UGO_FEC_RECONSTRUCT_DATA_ONLY, list, entries, s, rowoff, count);
  if (!st && max_rows)
    st = reconstruct_list_dev(c, shards, present, list, entries, groups, S, L, out, out_row_stride, 0,
                              UGO_FEC_RECONSTRUCT_DATA_ONLY, nullptr, s, rowoff, index,
                              static_cast<uint32_t>(max_rows));
  const int fr = scratch_free(c, scratch, s);
  return st ? st : fr;
}

int ugo_fec_reconstruct(ugo_fec* c, uint8_t* shards, const uint64_t* present, size_t groups, size_t S,
                        size_t pitch, unsigned flags, int8_t* status, void* stream) {
  if (!c) return UGO_FEC_ERR_INVALID_ARG;
  if (c->poisoned) return UGO_FEC_ERR_HIP;  // a service block that never left (svc_retire)
  if (pitch < S) return S == 0 ? UGO_FEC_ERR_SHARD_NO_DATA : UGO_FEC_ERR_INVALID_ARG;
  return ugo_fec_reconstruct_strided(c, shards, present, groups, S, pitch, size_t(c->n) * pitch, flags, status,
                                     stream);
}

int ugo_fec_reconstruct_rows(ugo_fec* c, const uint8_t* const* rows, const uint64_t* present, size_t groups,
                             size_t S, uint8_t* out, size_t out_row_stride, size_t out_group_stride, unsigned flags,
                             int8_t* status, void* stream) {
  if (!c) return UGO_FEC_ERR_INVALID_ARG;
  if (c->poisoned) return UGO_FEC_ERR_HIP;  // a service block that never left (svc_retire)
  if (S == 0) return UGO_FEC_ERR_SHARD_NO_DATA;
  if (groups == 0) return UGO_FEC_OK;
  if (S > 0xffffffffu || c->n > 64 || !rows || !present || !out) return UGO_FEC_ERR_INVALID_ARG;
  // output slots per group: p, or with DATA_ONLY min(d, p) (at most that many data rows are erased)
  const size_t oslots = (flags & UGO_FEC_RECONSTRUCT_DATA_ONLY) ? size_t(std::min(c->d, c->p)) : size_t(c->p);
  if (reinterpret_cast<uintptr_t>(out) % 16 || out_row_stride % 16 || out_group_stride % 16 ||
      !layout_disjoint(S, out_row_stride, oslots, out_group_stride, groups))
    return UGO_FEC_ERR_INVALID_ARG;
  DeviceGuard g(c->device);
  if (!g.ok) return UGO_FEC_ERR_NO_DEVICE;
  if (!device_view(rows) || !device_view(present) || !device_view(status) || !device_view(out))
    return UGO_FEC_ERR_INVALID_ARG;
  TimerScope ts(c);
  const hipStream_t s = static_cast<hipStream_t>(stream);
  const int mode = c->d_table ? 1 : 2;
  ugo::kern::Batch a = base_batch(c, nullptr, S, Layout{0, 0});
  a.rows = reinterpret_cast<const uint64_t*>(rows);
  a.n = static_cast<uint32_t>(c->n);
  a.out = out;
  a.ogstride = out_group_stride;
  a.orstride = out_row_stride;
  a.present = present;
  a.status = status;
  a.data_only = (flags & UGO_FEC_RECONSTRUCT_DATA_ONLY) ? 1u : 0u;
  a.chunks = static_cast<uint32_t>((S + 15) / 16);
  size_t per = slice_groups(a.chunks, true);
  uint8_t* work = nullptr;
  if (mode == 2) {
    per = std::min<size_t>(per, 65536);
    const int st = scratch_alloc(c, std::min(per, groups) * c->desc_stride + 64, s, reinterpret_cast<void**>(&work));
    if (st) return st;
  }
  struct Release {
    ugo_fec* c;
    uint8_t* p;
    hipStream_t s;
    ~Release() { (void)scratch_free(c, p, s); }
  } release{c, work, s};
  for (size_t g0 = 0; g0 < groups; g0 += per) {
    const size_t gn = std::min(per, groups - g0);
    a.g0 = g0;
    a.items = static_cast<uint32_t>(gn * a.chunks);
    if (mode == 1) {
      a.desc = c->d_table;
    } else {
      ugo::kern::Prep pr{};
      pr.desc = work;
      pr.present = present;
      pr.M = c->d_M;
      pr.gf_exp = c->d_gf;
      pr.gf_log = c->d_gf + 512;
      pr.g0 = g0;
      pr.g_desc0 = g0;
      pr.nmask = a.nmask;
      pr.desc_stride = c->desc_stride;
      pr.d = static_cast<uint32_t>(c->d);
      pr.n = static_cast<uint32_t>(c->n);
      pr.dpad = c->dpad;
      pr.epad = c->epad;
      if (ugo::kern::launch_prepare(pr, static_cast<uint32_t>(gn), s) != hipSuccess) return UGO_FEC_ERR_HIP;
      a.desc = work;
      a.g_desc0 = g0;
    }
    if (ugo::kern::launch_apply_rows(mode, a, s) != hipSuccess) return UGO_FEC_ERR_HIP;
  }
  return UGO_FEC_OK;
}

int ugo_fec_device_address(const ugo_fec* c, const void* p, void** dev) {
  if (!c || !dev) return UGO_FEC_ERR_INVALID_ARG;
  *dev = nullptr;
  DeviceGuard g(c->device);
  if (!g.ok) return UGO_FEC_ERR_NO_DEVICE;
  const uint8_t* q = static_cast<const uint8_t*>(p);
  if (!q || !device_view(q)) return UGO_FEC_ERR_INVALID_ARG;
  *dev = const_cast<uint8_t*>(q);
  return UGO_FEC_OK;
}

int ugo_fec_service_start(ugo_fec* c, unsigned idle_us) {
  if (!c) return UGO_FEC_ERR_INVALID_ARG;
  if (c->poisoned) return UGO_FEC_ERR_HIP;  // a service block that never left (svc_retire)
  DeviceGuard g(c->device);
  if (!g.ok) return UGO_FEC_ERR_NO_DEVICE;
  if (!c->svc_box) {
    void* p = nullptr;
    if (hipHostMalloc(&p, sizeof(ugo::kern::SvcBox), hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess)
      return UGO_FEC_ERR_HIP;
    std::memset(p, 0, sizeof(ugo::kern::SvcBox));
    c->svc_box = static_cast<ugo::kern::SvcBox*>(p);
    c->svc_dbox = c->svc_box;
    if (!device_view(c->svc_dbox)) return UGO_FEC_ERR_HIP;
  }
  if (!c->svc_stream) c->svc_stream = svc_lease(c);
  if (!c->svc_stream) {  // every service stream of the device is leased: the launch path serves this context
    c->svc_on = false;
    return UGO_FEC_OK;
  }
  int khz = 0;  // wall_clock64's rate (100 MHz on gfx950)
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, c->device) != hipSuccess || khz <= 0) khz = 100000;
  // at most 1 s resident after the last call: a process that exits without
  // ugo_fec_destroy leaves no long-running wave behind
  const uint64_t us = std::min<uint64_t>(idle_us ? idle_us : 2000u, 1000000u);
  c->svc_idle_ticks = us * uint64_t(khz) / 1000u;
  c->svc_khz = uint64_t(khz);
  c->svc_on = true;
  return UGO_FEC_OK;
}

int ugo_fec_service_stop(ugo_fec* c) {
  if (!c) return UGO_FEC_ERR_INVALID_ARG;
  if (c->poisoned) return UGO_FEC_ERR_HIP;
  DeviceGuard g(c->device);
  if (!g.ok) return UGO_FEC_ERR_NO_DEVICE;
  return svc_stop(c);
}

int ugo_fec_service_config(ugo_fec* c, unsigned timeout_ms, unsigned grace_ms, unsigned test_stall_us) {
  if (!c || test_stall_us > 10000000u) return UGO_FEC_ERR_INVALID_ARG;
  if (c->poisoned) return UGO_FEC_ERR_HIP;
  c->svc_timeout_ms = timeout_ms ? timeout_ms : 5000u;
  c->svc_grace_ms = grace_ms ? grace_ms : 5000u;
  c->svc_stall_us = test_stall_us;
  return UGO_FEC_OK;
}

int ugo_fec_poisoned(const ugo_fec* c) { return c && c->poisoned ? 1 : 0; }

#ifdef UGO_SVC_TRACE  // A/B builds only (tools/svc_trace.cpp): the last request's phase ticks
int ugo_fec_svc_trace(const ugo_fec* c, uint64_t* out) {
  if (!c || !c->svc_box || !out) return UGO_FEC_ERR_INVALID_ARG;
  for (int k = 0; k < 6; ++k) out[k] = reinterpret_cast<volatile const uint64_t*>(c->svc_box->trace)[k];
  return UGO_FEC_OK;
}
#endif

int ugo_fec_encode_host(ugo_fec* c, uint8_t* shards, size_t groups, size_t S, size_t pitch) {
  if (!c) return UGO_FEC_ERR_INVALID_ARG;
  if (c->poisoned) return UGO_FEC_ERR_HIP;  // a service block that never left (svc_retire)
  if (pitch < S) return S == 0 ? UGO_FEC_ERR_SHARD_NO_DATA : UGO_FEC_ERR_INVALID_ARG;
  int st = check_batch(c, shards, groups, S, interleaved(c, pitch));
  if (st || groups == 0 || c->p == 0) return st;
  DeviceGuard g(c->device);
  if (!g.ok) return UGO_FEC_ERR_NO_DEVICE;
  TimerScope ts(c);
  return host_path(c, shards, nullptr, groups, S, pitch, false, 0, nullptr);
}

int ugo_fec_reconstruct_host(ugo_fec* c, uint8_t* shards, const uint64_t* present, size_t groups, size_t S,
                             size_t pitch, unsigned flags, int8_t* status) {
  if (!c) return UGO_FEC_ERR_INVALID_ARG;
  if (c->poisoned) return UGO_FEC_ERR_HIP;  // a service block that never left (svc_retire)
  if (pitch < S) return S == 0 ? UGO_FEC_ERR_SHARD_NO_DATA : UGO_FEC_ERR_INVALID_ARG;
  int st = check_batch(c, shards, groups, S, interleaved(c, pitch));
  if (st || groups == 0) return st;
  if (!present) return UGO_FEC_ERR_INVALID_ARG;
  DeviceGuard g(c->device);
  if (!g.ok) return UGO_FEC_ERR_NO_DEVICE;
  TimerScope ts(c);
  return host_path(c, shards, present, groups, S, pitch, true, flags, status);
}

namespace {
// ugo_fec_rx_assemble / _frames: argument checks, device views, launch.  A
// frame row spans S + 6 bytes (the packet's header columns, then the payload).
int rx_assemble_abi(ugo_fec* c, const uint8_t* wire, size_t slot_stride, const uint16_t* lens, size_t npk,
                    const uint8_t* pad, uint64_t first_group, size_t groups, uint8_t* shards, size_t S,
                    size_t row_stride, size_t group_stride, uint64_t* present, uint32_t* stats, void* stream,
                    bool frame) {
  if (!c) return UGO_FEC_ERR_INVALID_ARG;
  if (c->poisoned) return UGO_FEC_ERR_HIP;  // a service block that never left (svc_retire)
  if (S == 0) return UGO_FEC_ERR_SHARD_NO_DATA;
  if (npk == 0) return UGO_FEC_OK;
  if (!wire || !lens || !shards || !present || groups == 0 || c->n > 64 || npk >= 0xffffffffull)
    return UGO_FEC_ERR_INVALID_ARG;
  if (slot_stride % 16 || slot_stride < 16 || reinterpret_cast<uintptr_t>(wire) % 16 ||
      reinterpret_cast<uintptr_t>(shards) % 16 || row_stride % 16 || group_stride % 16 ||
      (pad && reinterpret_cast<uintptr_t>(pad) % 16) || S > 0xffffffffu - 22)
    return UGO_FEC_ERR_INVALID_ARG;
  const size_t span = frame ? S + 6 : S;
  if (!layout_disjoint(span, row_stride, size_t(c->n), group_stride, groups)) return UGO_FEC_ERR_INVALID_ARG;
  DeviceGuard g(c->device);
  if (!g.ok) return UGO_FEC_ERR_NO_DEVICE;
  if (!device_view(wire) || !device_view(lens) || !device_view(pad) || !device_view(shards) ||
      !device_view(present) || !device_view(stats))
    return UGO_FEC_ERR_INVALID_ARG;
  TimerScope ts(c);
  return rx_assemble_dev(c, wire, slot_stride, lens, npk, pad, first_group, groups, shards, S, row_stride,
                         group_stride, present, stats, static_cast<hipStream_t>(stream), frame);
}
}  // namespace

int ugo_fec_rx_assemble(ugo_fec* c, const uint8_t* wire, size_t slot_stride, const uint16_t* lens, size_t npk,
                        const uint8_t* pad, uint64_t first_group, size_t groups, uint8_t* shards, size_t S,
                        size_t row_stride, size_t group_stride, uint64_t* present, uint32_t* stats,
                        void* stream) {
  return rx_assemble_abi(c, wire, slot_stride, lens, npk, pad, first_group, groups, shards, S, row_stride,
                         group_stride, present, stats, stream, false);
}

int ugo_fec_rx_assemble_frames(ugo_fec* c, const uint8_t* wire, size_t slot_stride, const uint16_t* lens,
                               size_t npk, const uint8_t* pad, uint64_t first_group, size_t groups, uint8_t* shards,
                               size_t S, size_t row_stride, size_t group_stride, uint64_t* present, uint32_t* stats,
                               void* stream) {
  return rx_assemble_abi(c, wire, slot_stride, lens, npk, pad, first_group, groups, shards, S, row_stride,
                         group_stride, present, stats, stream, true);
}

int ugo_fec_tx_assemble(ugo_fec* c, const uint8_t* pkts, size_t slot_in, const uint16_t* lens, size_t groups,
                        uint32_t first_seq, const uint8_t* pad, size_t max_len, uint8_t* wire, size_t slot_out,
                        uint16_t* wire_lens, int8_t* status, void* stream) {
  if (!c) return UGO_FEC_ERR_INVALID_ARG;
  if (c->poisoned) return UGO_FEC_ERR_HIP;  // a service block that never left (svc_retire)
  if (groups == 0) return UGO_FEC_OK;
  const uint64_t n = static_cast<uint64_t>(c->n);
  const uint32_t paws = static_cast<uint32_t>((0xffffffffull / n - 1) * n);  // ugo/fec.go:58
  const size_t need = round_up(max_len, 16);
  if (!pkts || !lens || !wire || !wire_lens || c->d > 32 || max_len < 6 || max_len > 0xffff ||
      slot_in % 16 || slot_out % 16 || slot_in < need || slot_out < need ||
      reinterpret_cast<uintptr_t>(pkts) % 16 || reinterpret_cast<uintptr_t>(wire) % 16 ||
      (pad && reinterpret_cast<uintptr_t>(pad) % 16) || first_seq % n || first_seq >= paws)
    return UGO_FEC_ERR_INVALID_ARG;
  DeviceGuard g(c->device);
  if (!g.ok) return UGO_FEC_ERR_NO_DEVICE;
  if (!device_view(pkts) || !device_view(lens) || !device_view(pad) || !device_view(wire) ||
      !device_view(wire_lens) || !device_view(status))
    return UGO_FEC_ERR_INVALID_ARG;
  TimerScope ts(c);
  ugo::kern::TxArgs a{};
  a.pkts = pkts;
  a.lens = lens;
  a.pad = pad;
  a.desc = c->d_encdesc;
  a.wire = wire;
  a.wire_lens = wire_lens;
  a.status = status;
  a.slot_in = slot_in;
  a.slot_out = slot_out;
  a.first_seq = first_seq;
  a.paws = paws;
  a.max_len = static_cast<uint32_t>(max_len);
  a.chunks = static_cast<uint32_t>(need / 16);
  a.d = static_cast<uint32_t>(c->d);
  a.p = static_cast<uint32_t>(c->p);
  a.dpad = c->dpad;
  a.epad = c->epad;
  const int dmax = ugo::kern::has_const_encode(c->d, c->p) ? 0 : ugo::kern::apply_dmax(c->d);
  const uint64_t per_launch = (1ull << 31) / a.chunks;  // items of one launch fit 32 bits
  for (uint64_t g0 = 0; g0 < groups; g0 += per_launch) {
    a.g0 = g0;
    a.groups = std::min<uint64_t>(per_launch, groups - g0);
    const int st = hip_status(ugo::kern::launch_tx_assemble(dmax, a, static_cast<hipStream_t>(stream)));
    if (st != UGO_FEC_OK) return st;
  }
  return UGO_FEC_OK;
}

// ---- host-memory RX and TX paths ---------------------------
// The whole RX path from host memory to host memory: a received packet ring in
// pinned memory (a recvmmsg batch) is copied to the device in chunks on one
// copy stream, each chunk assembled (rx_assemble_dev, one call per chunk into
// one batch: first copy wins across the calls) on a second stream as soon as its
// copy lands, so copies and kernels overlap; then the lossy-group list, the
// data-only Reconstruct of those groups into a row-compact output (the
// `recovered` list of ugo/fec.go:203-207), and the D2H of those rows only.
// The host RX path's batch layout: payload rows (0, the default) or frame rows
// (1, ugo_fec_rx_assemble_frames).  Measured the same end to end (22.7 ms for
// the bench's ring either way, the call being PCIe-bound:
// profiles/r6/host_rx/frames_vs_payload.jsonl); with both place kernels at 3
// blocks per CU the two placements tie on the device (frames 1 % ahead in order
// on the mean of four runs, 4 % either way box to box), and
// payload rows need no row shift before the D2H.
#ifndef UGO_RX_FRAMES
#define UGO_RX_FRAMES 0
#endif
constexpr bool kRxFrames = UGO_RX_FRAMES != 0;
#ifndef UGO_RX_STAGE_MIB
#define UGO_RX_STAGE_MIB 64
#endif
constexpr size_t kRxStageBytes = size_t(UGO_RX_STAGE_MIB) << 20;  // ring bytes per H2D copy at most

int ugo_fec_rx_recover_host(ugo_fec* c, const uint8_t* wire, size_t slot_stride, const uint16_t* lens, size_t npk,
                            const uint8_t* pad, uint64_t first_group, size_t groups, size_t S, uint64_t* present_out,
                            uint32_t* stats_out, uint8_t* out, size_t out_row_stride, size_t max_out,
                            uint32_t* out_index, size_t* n_out) {
  if (!c || !n_out) return UGO_FEC_ERR_INVALID_ARG;
  *n_out = 0;
  if (c->poisoned) return UGO_FEC_ERR_HIP;  // a service block that never left (svc_retire)
  if (S == 0) return UGO_FEC_ERR_SHARD_NO_DATA;
  if (groups == 0) return UGO_FEC_OK;
  if ((npk && (!wire || !lens)) || c->n > 16 || !c->d_table || groups * size_t(c->n) >= 0xffffffffull || npk >= 0xffffffffull ||
      slot_stride % 16 || slot_stride < 16 || S > 0xffffffffu - 22 || out_row_stride < S ||
      (max_out && (!out || !out_index)))
    return UGO_FEC_ERR_INVALID_ARG;
  DeviceGuard g(c->device);
  if (!g.ok) return UGO_FEC_ERR_NO_DEVICE;
  TimerScope ts(c);
  int st = ensure_streams(c);
  if (st) return st;
  const hipStream_t s0 = c->streams[0];  // assembly and recovery; copies on streams[1]
  // with frame rows (kRxFrames, ugo_fec_rx_assemble_frames) each row holds its decrypted packet, the
  // payload at column 6; the recovery then runs over the frame window (GF columns are independent) and
  // only the payload columns of a recovered row come back
  const size_t fo = kRxFrames ? 6 : 0, FS = S + fo;
  // (frame rows at a 64-B pitch: whole 64-B lines per row, rx_frame_fill)
  const size_t n = size_t(c->n), pitch = round_up(FS, kRxFrames ? 64 : 16), slots = size_t(std::min(c->d, c->p));
  // packets per chunk: at most a kRxStageBytes stage, at least 4 chunks so copies and assembly overlap,
  // and at most 32 chunks (the chunks grow with the ring past that: see kTxMaxChunks)
  const size_t cpk =
      std::max<size_t>({size_t(1), (npk + 31) / 32, std::min((npk + 3) / 4, kRxStageBytes / slot_stride)});
  const size_t stage_bytes = round_up(cpk * slot_stride, 256);
  // every recovered row fits: a recoverable group rebuilds at most min(d, p) data rows
  const size_t max_rows = max_out ? groups * slots : 1;
  // one scratch block: batch | present | list | row offsets | counts, stats | row ids | rows | pad | lens | ring stages
  size_t off = 0;
  auto take = [&](size_t bytes) { const size_t o = off; off = round_up(off + bytes, 256); return o; };
  // (+ the chunk calls' rx_assemble scratch, shared: they run in order on s0; + frame rows: the
  // recovered rows shifted to payload rows at a 16-B pitch for the D2H)
  const size_t opitch = round_up(S, 16);
  const size_t o_batch = take(n * groups * pitch), o_pres = take(groups * 8), o_list = take(groups * 4),
               o_roff = take(groups * 4), o_ctl = take(64), o_rid = take(max_rows * 4), o_out = take(max_rows * pitch),
               o_pad = take(pad ? slot_stride : 16), o_lens = take(std::max<size_t>(npk, 1) * 2),
               o_rxs = take(rx_scratch_bytes(c, groups)), o_pk = take(kRxFrames ? max_rows * opitch : 16),
               o_stage = take(kRxStages * stage_bytes);
  uint8_t* base = nullptr;
  st = scratch_alloc(c, off, s0, reinterpret_cast<void**>(&base));
  if (st) return st;
  struct Release {  // the copy streams finish before the scratch goes back (also on an early return)
    ugo_fec* c;
    uint8_t* p;
    hipStream_t s;
    ~Release() {
      (void)hipStreamSynchronize(c->streams[1]);
      (void)hipStreamSynchronize(c->streams[2]);
      (void)scratch_free(c, p, s);
    }
  } release{c, base, s0};
  uint8_t* batch = base + o_batch;
  uint64_t* dpres = reinterpret_cast<uint64_t*>(base + o_pres);
  uint32_t* dlist = reinterpret_cast<uint32_t*>(base + o_list);
  uint32_t* droff = reinterpret_cast<uint32_t*>(base + o_roff);
  uint32_t* dcount = reinterpret_cast<uint32_t*>(base + o_ctl);  // [0] lossy groups, [1] recovered rows
  uint32_t* dstats = dcount + 4;
  uint32_t* drid = reinterpret_cast<uint32_t*>(base + o_rid);
  uint8_t* dout = base + o_out;
  uint8_t* dpad = pad ? base + o_pad : nullptr;
  uint16_t* dlens = reinterpret_cast<uint16_t*>(base + o_lens);
  // ev[b]: stage b's copy landed; ev[kRxStages + b]: its assembly is done (the stage is free)
  hipEvent_t ev[2 * kRxStages] = {};
  struct Events {
    hipEvent_t* e;
    ~Events() {
      for (int i = 0; i < 2 * kRxStages; ++i)
        if (e[i]) (void)hipEventDestroy(e[i]);
    }
  } evs{ev};
  for (int i = 0; i < 2 * kRxStages; ++i)
    if (hipEventCreateWithFlags(&ev[i], hipEventDisableTiming) != hipSuccess) return UGO_FEC_ERR_HIP;
  if (hipMemsetAsync(dpres, 0, groups * 8, s0) != hipSuccess || hipMemsetAsync(dcount, 0, 64, s0) != hipSuccess ||
      (pad && hipMemcpyAsync(dpad, pad, slot_stride, hipMemcpyHostToDevice, s0) != hipSuccess))
    return UGO_FEC_ERR_HIP;
  // the copy streams start after the zeroing (their stages are this call's scratch)
  for (int b = 0; b < kRxStages; ++b)
    if (hipEventRecord(ev[kRxStages + b], s0) != hipSuccess) return UGO_FEC_ERR_HIP;
  // all the lengths in one copy ahead of the first stage (a small copy between two ring copies on a
  // stream cost a ~0.1-ms gap per chunk: profiles/r5/host_rx_trace)
  if (npk && (hipStreamWaitEvent(c->streams[1], ev[kRxStages], 0) != hipSuccess ||
              hipMemcpyAsync(dlens, lens, npk * sizeof(uint16_t), hipMemcpyHostToDevice, c->streams[1]) != hipSuccess))
    return UGO_FEC_ERR_HIP;
  // copies run up to kRxStages - 1 chunks ahead of the assembly in enqueue order too, so a host
  // thread held up between two chunks does not leave the link idle
  const size_t nchunks = (npk + cpk - 1) / cpk;
  size_t next = 0;
  for (size_t k = 0; k < nchunks; ++k) {
    for (; next < nchunks && next < k + kRxStages; ++next) {
      const int b = static_cast<int>(next % kRxStages);
      // every ring copy on streams[1]: 23.4-24.2 ms over six process histories (23.1-23.2 with the
      // low-priority copy queue), against 22.3-25.0 alternating streams 1 and 2
      // (profiles/r5/host_tx_route/host_rx_copy_streams_*.jsonl, host_tx_normal_2stream.jsonl)
      const hipStream_t cs = c->streams[1];
      const size_t p0 = next * cpk, m = std::min(cpk, npk - p0);
      if (hipStreamWaitEvent(cs, ev[kRxStages + b], 0) != hipSuccess ||
          hipMemcpyAsync(base + o_stage + b * stage_bytes, wire + p0 * slot_stride, m * slot_stride,
                         hipMemcpyHostToDevice, cs) != hipSuccess ||
          hipEventRecord(ev[b], cs) != hipSuccess)
        return UGO_FEC_ERR_HIP;
    }
    const int b = static_cast<int>(k % kRxStages);
    const size_t p0 = k * cpk, m = std::min(cpk, npk - p0);
    if (hipStreamWaitEvent(s0, ev[b], 0) != hipSuccess) return UGO_FEC_ERR_HIP;
    // (chunk 0's wait covers the lengths' copy, earlier on the same stream; later chunks follow it on s0)
    st = rx_assemble_dev(c, base + o_stage + b * stage_bytes, slot_stride, dlens + p0, m, dpad, first_group, groups,
                         batch, S, groups * pitch, pitch, dpres, dstats, s0, kRxFrames, base + o_rxs);
    if (st) return st;
    if (hipEventRecord(ev[kRxStages + b], s0) != hipSuccess) return UGO_FEC_ERR_HIP;
  }
  // the lossy groups and, per entry, where its rows start in the row-compact output
  st = lossy_list_dev(c, dpres, groups, UGO_FEC_RECONSTRUCT_DATA_ONLY, dlist, dcount, s0, droff, dcount + 1);
  if (st) return st;
  if (max_out) {
    st = reconstruct_list_dev(c, batch, dpres, dlist, dcount, groups, FS, Layout{groups * pitch, pitch}, dout, pitch,
                              0, UGO_FEC_RECONSTRUCT_DATA_ONLY, nullptr, s0, droff, drid);
    if (st) return st;
  }
  uint32_t hcnt[8] = {};
  if (hipMemcpyAsync(hcnt, dcount, 32, hipMemcpyDeviceToHost, s0) != hipSuccess || hipStreamSynchronize(s0) != hipSuccess)
    return UGO_FEC_ERR_HIP;
  const size_t total = hcnt[1], w = std::min<size_t>(total, max_out);
  *n_out = total;
  hipError_t e = hipSuccess;
  if (w) {  // only the recovered rows cross PCIe: w rows of S bytes
    e = hipMemcpyAsync(out_index, drid, w * 4, hipMemcpyDeviceToHost, s0);
    const uint8_t* rows = dout;
    size_t rpitch = pitch;
    if (kRxFrames && e == hipSuccess) {
      // frame rows -> 16-B aligned payload rows first: a 2-D copy from rows at column 6 ran as the
      // runtime's copyBufferRect kernel at ~16 GB/s (2.75 ms for 32k rows, profiles/r6/host_rx_trace),
      // from aligned rows it is a DMA copy at the link's rate
      e = ugo::kern::launch_shift_rows(dout, pitch, static_cast<uint32_t>(fo), base + o_pk, opitch,
                                       static_cast<uint32_t>(S), w, s0);
      rows = base + o_pk;
      rpitch = opitch;
    }
    if (e == hipSuccess) e = hipMemcpy2DAsync(out, out_row_stride, rows, rpitch, S, w, hipMemcpyDeviceToHost, s0);
  }
  if (e == hipSuccess && present_out) e = hipMemcpyAsync(present_out, dpres, groups * 8, hipMemcpyDeviceToHost, s0);
  if (e == hipSuccess && stats_out) e = hipMemcpyAsync(stats_out, dstats, 20, hipMemcpyDeviceToHost, s0);
  if (e == hipSuccess) e = hipStreamSynchronize(s0);
  return hip_status(e);
}

// The TX path from host memory to host memory: groups in chunks through
// kTxStages device stages -- the data packets' H2D on streams[1], tx_assemble
// and then the wire packets' D2H on streams[0] -- joined by events, so the two
// copy directions run at once (with the low-priority copy queue, a third stream
// for the D2H copies ran 25.9-28.6 ms over six process histories, the D2H
// behind the kernel on its stream 26.5-26.6 in all six,
// profiles/r5/host_tx_route/host_tx_d2h_stream.jsonl); the lengths go in with
// one copy ahead of the first chunk and the wire lengths and statuses come back
// with one copy after the last (a
// small copy between two large ones costs the engine ~0.1 ms,
// profiles/r5/host_rx_trace).  Round 5's first form (H2D -> kernel -> D2H per
// chunk on three round-robin streams, a stream's next input behind its
// previous output) took 30.6 ms for 65,536 (10+3) groups (tools/host_txrx_ab.py,
// profiles/r5/host_txrx_ab.jsonl); the kernel reading the pinned data packets
// through their mapping instead of the H2D copies, 40.1-40.3 ms
// (profiles/r5/host_tx_route_ab.md).
#ifndef UGO_TX_STAGES
#define UGO_TX_STAGES 4
#endif
constexpr int kTxStages = UGO_TX_STAGES;
#ifndef UGO_TX_CHUNK_MIB
#define UGO_TX_CHUNK_MIB 64
#endif
constexpr size_t kTxChunkBytes = size_t(UGO_TX_CHUNK_MIB) << 20;  // a stage's input + output bytes at most
// At most kTxMaxChunks chunks per call: the chunks grow with the batch past
// that.  Calls of more chunks ran 2-4x slower, with everything enqueued at once
// (64-MiB chunks at 65,536 / 131,072 / 262,144 groups: 26.7 / 52-130 / 210 ms;
// 32-MiB chunks at 65,536: 48-54 ms); bounding the enqueue from the host
// (waiting for chunk k - 16 or k - 8 before enqueueing chunk k) was slower
// still (42 / 122 / 249 ms), and so was spreading each copy direction over
// two streams (43.7 ms at 65,536) -- profiles/r5/host_tx_chunk_ab*.jsonl.
#ifndef UGO_TX_MAX_CHUNKS
#define UGO_TX_MAX_CHUNKS 32
#endif
constexpr size_t kTxMaxChunks = UGO_TX_MAX_CHUNKS;

// The wire packets leave through the stage and a D2H copy behind the kernel
// (route 0), or, pinned by ugo_fec_set_tx_host_route, written by the kernel
// itself through the pinned wire buffer's device mapping (route 1, no D2H
// copy: 30.4 ms for 65,536 (10+3) groups against 26.0-27.6,
// profiles/r5/host_tx_route_ab.md).  An unmapped (pageable) or unaligned wire
// buffer takes route 0.

int ugo_fec_tx_assemble_host(ugo_fec* c, const uint8_t* pkts, size_t slot_in, const uint16_t* lens, size_t groups,
                             uint32_t first_seq, const uint8_t* pad, size_t max_len, uint8_t* wire, size_t slot_out,
                             uint16_t* wire_lens, int8_t* status) {
  if (!c) return UGO_FEC_ERR_INVALID_ARG;
  if (c->poisoned) return UGO_FEC_ERR_HIP;  // a service block that never left (svc_retire)
  if (groups == 0) return UGO_FEC_OK;
  const uint64_t n = static_cast<uint64_t>(c->n), d = static_cast<uint64_t>(c->d);
  const uint32_t paws = static_cast<uint32_t>((0xffffffffull / n - 1) * n);  // ugo/fec.go:58
  const size_t need = round_up(max_len, 16);
  if (!pkts || !lens || !wire || !wire_lens || c->d > 32 || max_len < 6 || max_len > 0xffff || slot_in % 16 ||
      slot_out % 16 || slot_in < need || slot_out < need || first_seq % n || first_seq >= paws)
    return UGO_FEC_ERR_INVALID_ARG;
  DeviceGuard g(c->device);
  if (!g.ok) return UGO_FEC_ERR_NO_DEVICE;
  TimerScope ts(c);
  int st = ensure_streams(c);
  if (st) return st;
  const hipStream_t sk = c->streams[0], sin = c->streams[1];
  const size_t per_group = d * slot_in + n * slot_out;
  uint8_t* zwire = wire;  // route 1: the wire buffer's device view, 16-B aligned
  const int route =
      c->tx_route == 1 && device_view(zwire) && reinterpret_cast<uintptr_t>(zwire) % 16 == 0 ? 1 : 0;
  // groups per chunk: a stage of at most kTxChunkBytes, at least 8 chunks so the two directions
  // overlap, at most kTxMaxChunks
  const size_t cg = std::max<size_t>({size_t(1), (groups + kTxMaxChunks - 1) / kTxMaxChunks,
                                      std::min((groups + 7) / 8, kTxChunkBytes / per_group)});
  // scratch: lengths [groups][d] | wire lengths [groups][n] | statuses [groups] | keystream | stages
  size_t off = 0;
  auto take = [&](size_t bytes) { const size_t o = off; off = round_up(off + bytes, 256); return o; };
  const size_t o_lens = take(groups * d * 2), o_wl = take(groups * n * 2), o_st = take(groups),
               o_pad = take(pad ? need : 16), o_stages = off;
  const size_t o_in = 0, o_wire = round_up(cg * d * slot_in, 256), stage_bytes = o_wire + round_up(cg * n * slot_out, 256);
  uint8_t* base = nullptr;
  st = scratch_alloc(c, o_stages + size_t(kTxStages) * stage_bytes, sk, reinterpret_cast<void**>(&base));
  if (st) return st;
  constexpr int kEv = 2 * kTxStages + 1;  // in[b] | out[b] (stage free) | ready
  hipEvent_t ev[kEv] = {};
  struct Release {  // the copy streams finish before the scratch goes back (also on an early return)
    ugo_fec* c;
    uint8_t* p;
    hipEvent_t* e;
    ~Release() {
      (void)hipStreamSynchronize(c->streams[1]);
      (void)hipStreamSynchronize(c->streams[2]);
      (void)scratch_free(c, p, c->streams[0]);
      for (int i = 0; i < kEv; ++i)
        if (e[i]) (void)hipEventDestroy(e[i]);
    }
  } release{c, base, ev};
  for (int i = 0; i < kEv; ++i)
    if (hipEventCreateWithFlags(&ev[i], hipEventDisableTiming) != hipSuccess) return UGO_FEC_ERR_HIP;
  uint16_t* dlens = reinterpret_cast<uint16_t*>(base + o_lens);
  uint16_t* dwl = reinterpret_cast<uint16_t*>(base + o_wl);
  int8_t* dst = reinterpret_cast<int8_t*>(base + o_st);
  uint8_t* dpad = pad ? base + o_pad : nullptr;
  if ((pad && hipMemcpyAsync(dpad, pad, need, hipMemcpyHostToDevice, sk) != hipSuccess) ||
      hipEventRecord(ev[2 * kTxStages], sk) != hipSuccess ||  // the scratch is this call's from here on
      hipStreamWaitEvent(sin, ev[2 * kTxStages], 0) != hipSuccess ||
      hipMemcpyAsync(dlens, lens, groups * d * 2, hipMemcpyHostToDevice, sin) != hipSuccess)
    return UGO_FEC_ERR_HIP;
  ugo::kern::TxArgs a{};
  a.desc = c->d_encdesc;
  a.slot_in = slot_in;
  a.slot_out = slot_out;
  a.paws = paws;
  a.max_len = static_cast<uint32_t>(max_len);
  a.chunks = static_cast<uint32_t>(need / 16);
  a.d = static_cast<uint32_t>(c->d);
  a.p = static_cast<uint32_t>(c->p);
  a.dpad = c->dpad;
  a.epad = c->epad;
  a.pad = dpad;
  const int dmax = ugo::kern::has_const_encode(c->d, c->p) ? 0 : ugo::kern::apply_dmax(c->d);
  size_t k = 0;
  for (size_t g0 = 0; g0 < groups; g0 += cg, ++k) {
    const size_t gn = std::min(cg, groups - g0);
    const int b = static_cast<int>(k % kTxStages);
    uint8_t* sb = base + o_stages + b * stage_bytes;
    // input: the stage's previous output (chunk k - kTxStages) must have left; chunk 0's event also
    // covers the lengths, copied before it on the same stream
    if ((k >= size_t(kTxStages) && hipStreamWaitEvent(sin, ev[kTxStages + b], 0) != hipSuccess) ||
        hipMemcpyAsync(sb + o_in, pkts + g0 * d * slot_in, gn * d * slot_in, hipMemcpyHostToDevice, sin) !=
            hipSuccess ||
        hipEventRecord(ev[b], sin) != hipSuccess || hipStreamWaitEvent(sk, ev[b], 0) != hipSuccess)
      return UGO_FEC_ERR_HIP;
    a.pkts = sb + o_in;
    a.lens = dlens + g0 * d;
    a.wire = route == 1 ? zwire + g0 * n * slot_out : sb + o_wire;
    a.wire_lens = dwl + g0 * n;
    a.status = status ? dst + g0 : nullptr;
    a.first_seq = static_cast<uint32_t>((uint64_t(first_seq) + uint64_t(g0) * n) % paws);
    a.g0 = 0;
    a.groups = gn;
    // the wire packets out behind the kernel on its stream (route 1: already written); the stage
    // is free after that
    if (ugo::kern::launch_tx_assemble(dmax, a, sk) != hipSuccess ||
        (route == 0 && hipMemcpyAsync(wire + g0 * n * slot_out, sb + o_wire, gn * n * slot_out,
                                      hipMemcpyDeviceToHost, sk) != hipSuccess) ||
        hipEventRecord(ev[kTxStages + b], sk) != hipSuccess)
      return UGO_FEC_ERR_HIP;
  }
  // the wire lengths and statuses of every chunk: one copy each, behind the last chunk's kernel
  if (hipMemcpyAsync(wire_lens, dwl, groups * n * 2, hipMemcpyDeviceToHost, sk) != hipSuccess ||
      (status && hipMemcpyAsync(status, dst, groups, hipMemcpyDeviceToHost, sk) != hipSuccess))
    return UGO_FEC_ERR_HIP;
  for (int i = 0; i < kStreams; ++i)
    if (hipStreamSynchronize(c->streams[i]) != hipSuccess) return UGO_FEC_ERR_HIP;
  return UGO_FEC_OK;
}

int ugo_fec_set_host_copy_queue(ugo_fec* c, int on) {
  if (!c || (on != 0 && on != 1)) return UGO_FEC_ERR_INVALID_ARG;
  if (c->poisoned) return UGO_FEC_ERR_HIP;
  if (c->host_copy_queue == (on == 1)) return UGO_FEC_OK;
  DeviceGuard g(c->device);
  if (!g.ok) return UGO_FEC_ERR_NO_DEVICE;
  if (c->streams[1]) {  // made again, from the other class, at the next host-path call
    if (hipStreamSynchronize(c->streams[1]) != hipSuccess ||
        (!is_shared_stream(c, 1) && hipStreamDestroy(c->streams[1]) != hipSuccess))
      return UGO_FEC_ERR_HIP;
    c->streams[1] = nullptr;
    c->streams_shared = false;
  }
  c->host_copy_queue = on == 1;
  return UGO_FEC_OK;
}

int ugo_fec_set_tx_host_route(ugo_fec* c, int route) {
  if (!c || route < 0 || route > 1) return UGO_FEC_ERR_INVALID_ARG;
  c->tx_route = route;
  return UGO_FEC_OK;
}

int ugo_fec_packet_decode(ugo_fec* c, const uint8_t* pkts, size_t slot, const uint16_t* lens, size_t npk,
                          const uint8_t* pad, unsigned flags, ugo_pkt_info* info, uint64_t* ranges,
                          size_t max_ranges, ugo_pkt_segment* segs, size_t max_segments, void* stream) {
  static_assert(sizeof(ugo_pkt_info) == 64, "ugo_pkt_info is 64 bytes");
  static_assert(sizeof(ugo_pkt_segment) == 16, "ugo_pkt_segment is 16 bytes");
  if (!c) return UGO_FEC_ERR_INVALID_ARG;
  if (c->poisoned) return UGO_FEC_ERR_HIP;  // a service block that never left (svc_retire)
  if (npk == 0) return UGO_FEC_OK;
  if (!pkts || !lens || !info || slot % 16 || slot == 0 || slot > 0xffff ||
      reinterpret_cast<uintptr_t>(pkts) % 16 || (pad && reinterpret_cast<uintptr_t>(pad) % 16) ||
      (max_ranges && !ranges) || (max_segments && !segs) || max_ranges > 0xffff || max_segments > 0xffff ||
      (flags & ~UGO_PKT_FEC_FRAMED))
    return UGO_FEC_ERR_INVALID_ARG;
  DeviceGuard g(c->device);
  if (!g.ok) return UGO_FEC_ERR_NO_DEVICE;
  if (!device_view(pkts) || !device_view(lens) || !device_view(pad) || !device_view(info) ||
      !device_view(ranges) || !device_view(segs))
    return UGO_FEC_ERR_INVALID_ARG;
  TimerScope ts(c);
  ugo::kern::PktArgs a{};
  a.pkts = pkts;
  a.lens = lens;
  a.pad = pad;
  a.info = info;
  a.ranges = ranges;
  a.segs = segs;
  a.npk = npk;
  a.slot = slot;
  a.max_ranges = static_cast<uint32_t>(max_ranges);
  a.max_segments = static_cast<uint32_t>(max_segments);
  a.framed = flags & UGO_PKT_FEC_FRAMED;
  return hip_status(ugo::kern::launch_packet_decode(a, static_cast<hipStream_t>(stream)));
}

int ugo_fec_rc4_keystream(const uint8_t* key, size_t key_len, uint8_t* out, size_t n) {
  if (!key || key_len == 0 || key_len > 256 || (n && !out)) return UGO_FEC_ERR_INVALID_ARG;
  ugo::rc4_keystream(key, key_len, out, n);
  return UGO_FEC_OK;
}

int ugo_fec_timing_begin(ugo_fec* c, size_t max_launches) {
  if (c && c->poisoned) return UGO_FEC_ERR_HIP;
  if (!c || max_launches == 0 || max_launches > (size_t(1) << 20)) return UGO_FEC_ERR_INVALID_ARG;
  DeviceGuard g(c->device);
  if (!g.ok) return UGO_FEC_ERR_NO_DEVICE;
  timer_release(c);
  ugo::kern::LaunchTimer& t = c->timer;
  t.ev = new (std::nothrow) hipEvent_t[2 * max_launches]();
  t.kid = new (std::nothrow) uint32_t[max_launches]();
  if (!t.ev || !t.kid) {
    timer_release(c);
    return UGO_FEC_ERR_INVALID_ARG;
  }
  t.cap = max_launches;
  for (size_t i = 0; i < 2 * max_launches; ++i)
    if (hipEventCreate(&t.ev[i]) != hipSuccess) {
      timer_release(c);
      return UGO_FEC_ERR_HIP;
    }
  c->timing = true;
  return UGO_FEC_OK;
}

int ugo_fec_timing_end(ugo_fec* c, ugo_fec_launch_time* out, size_t cap, size_t* n_out, size_t* n_untimed) {
  if (!c || (cap && !out)) return UGO_FEC_ERR_INVALID_ARG;
  DeviceGuard g(c->device);
  if (!g.ok) return UGO_FEC_ERR_NO_DEVICE;
  ugo::kern::LaunchTimer& t = c->timer;
  int st = UGO_FEC_OK;
  size_t n = 0;
  for (size_t i = 0; i < t.used; ++i) {
    if (hipEventSynchronize(t.ev[2 * i + 1]) != hipSuccess) {
      st = UGO_FEC_ERR_HIP;
      break;
    }
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, t.ev[2 * i], t.ev[2 * i + 1]) != hipSuccess) {
      st = UGO_FEC_ERR_HIP;
      break;
    }
    if (n < cap) out[n++] = ugo_fec_launch_time{t.kid[i], ms};
  }
  if (n_out) *n_out = n;
  if (n_untimed) *n_untimed = t.dropped;
  timer_release(c);
  return st;
}

// Fault injection for tests (ugo_fec_set_host_alloc_limit): pinned
// allocations larger than the limit fail, as on a host out of pinnable memory.
// An explicit call rather than an environment variable read on the allocation
// path (a stray variable in deployment would fail every allocation
// silently, and getenv races a concurrent setenv).
static std::atomic<unsigned long long> g_host_alloc_limit{0};

int ugo_fec_set_host_alloc_limit(size_t bytes) {
  g_host_alloc_limit.store(bytes, std::memory_order_relaxed);
  return UGO_FEC_OK;
}

int ugo_fec_host_alloc(size_t bytes, void** out) {
  if (!out) return UGO_FEC_ERR_INVALID_ARG;
  *out = nullptr;
  const unsigned long long lim = g_host_alloc_limit.load(std::memory_order_relaxed);
  if (lim && bytes > lim) return UGO_FEC_ERR_HIP;
  return hip_status(hipHostMalloc(out, bytes ? bytes : 1, hipHostMallocDefault));
}

int ugo_fec_host_free(void* p) { return hip_status(hipHostFree(p)); }

}  // extern "C"
