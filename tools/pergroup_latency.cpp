// pergroup_latency.cpp -- per-call cost of the drop-in per-group path (the
// "unchanged signatures" route: ugo calls Encode once per group from calcECC,
// ugo/fec.go:238, and Reconstruct once per lossy group from input, :202, via
// Conn.handlePacket ugo/conn.go:392-400), measured through the C-ABI only
// (include/ugo_fec.h, include/ugo_fec_conn.h), on the GPU box.
//
//   calc_ecc        ugo_fecconn_calc_ecc, 13 x 1476-B buffers, window [6, 1476)
//   encode_host_g1  ugo_fec_encode_host, one pinned group (10+3) x 1470
//   input_lossless  the 13 ugo_fecconn_input calls of a group with no loss
//   input_lossy     the 12 ugo_fecconn_input calls of a group missing one data
//                   shard (the 11th triggers Reconstruct on the GPU)
//   input_batch_B   the same lossy stream with ugo_fecconn_set_batch(B):
//                   one launch per B lossy groups, flush included
//   input_batch_B_overlap  the same with UGO_FECCONN_BATCH_OVERLAP (each batch
//                   recovered while the next fills), flush included
//   shim_*          the cgo shim of INTEGRATION.md §2, call for call (GoShim
//                   below: check_shards, copy into the pinned stage at the
//                   16-B pitch, *_host with groups = 1, copy out): Encode of a
//                   1470-B calcECC window, Reconstruct / ReconstructData of a
//                   1476-B input group with one lost data shard
//
// Prints one JSON line per case: median / p10 / p90 microseconds per group
// (per call for calc_ecc and encode_host_g1) over `reps` repetitions.
// Build: make -C tools pergroup_latency (links ugo_amd/libugofec.so).
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "../include/ugo_fec.h"
#include "../include/ugo_fec_conn.h"

namespace {

using clk = std::chrono::steady_clock;
constexpr int D = 10, P = 3, N = 13, RXLIMIT = 128;
constexpr size_t PKT = UGO_FEC_MAX_PACKET;

double us_since(clk::time_point t0) {
  return std::chrono::duration<double, std::micro>(clk::now() - t0).count();
}

void report(const char* name, std::vector<double> v, const char* unit, double extra = -1.0, double mean = -1.0) {
  std::sort(v.begin(), v.end());
  const auto q = [&](double f) { return v[std::min(v.size() - 1, static_cast<size_t>(f * v.size()))]; };
  std::printf("{\"case\": \"%s\", \"median_us\": %.3f, \"p10_us\": %.3f, \"p90_us\": %.3f, \"unit\": \"%s\", \"reps\": %zu",
              name, q(0.5), q(0.1), q(0.9), unit, v.size());
  if (extra >= 0) std::printf(", \"groups_per_rep\": %.0f", extra);
  if (mean >= 0) std::printf(", \"mean_us\": %.3f", mean);
  std::printf("}\n");
  std::fflush(stdout);
}

void check(int st, const char* what) {
  if (st != UGO_FEC_OK) {
    std::fprintf(stderr, "%s: %s\n", what, ugo_fec_strerror(st));
    std::exit(1);
  }
}

// Wire packets of `groups` groups starting at seqid base; shard `drop` of
// every group is left out (drop < 0: none).
std::vector<std::vector<uint8_t>> stream(uint32_t base, int groups, int drop, std::mt19937& rng) {
  std::vector<std::vector<uint8_t>> out;
  for (int g = 0; g < groups; ++g)
    for (int k = 0; k < N; ++k) {
      if (k == drop) continue;
      std::vector<uint8_t> w(PKT);
      const uint32_t seq = base + static_cast<uint32_t>(g * N + k);
      std::memcpy(w.data(), &seq, 4);
      const uint16_t flag = k < D ? UGO_FEC_TYPE_DATA : UGO_FEC_TYPE_FEC;
      std::memcpy(w.data() + 4, &flag, 2);
      for (size_t i = 6; i < PKT; ++i) w[i] = static_cast<uint8_t>(rng());
      out.push_back(std::move(w));
    }
  return out;
}

// INTEGRATION.md §2's Go shim in C++, statement for statement (Go slices ->
// std::vector; a nil / empty shard -> an empty vector).
struct GoShim {
  ugo_fec* ctx = nullptr;
  int d = 0, p = 0;
  void* stage = nullptr;
  size_t stageN = 0;
  static size_t pitch(size_t S) { return (S + 15) & ~size_t(15); }
  uint8_t* staging(size_t n) {
    if (n > stageN) {
      if (stage) ugo_fec_host_free(stage);
      ugo_fec_host_alloc(n, &stage);
      stageN = n;
    }
    return static_cast<uint8_t*>(stage);
  }
  int check(const std::vector<std::vector<uint8_t>>& shards, bool nilOK, size_t* S) {
    const int n = d + p;
    if (static_cast<int>(shards.size()) != n) return UGO_FEC_ERR_TOO_FEW_SHARDS;
    std::vector<size_t> lens(n);
    for (int i = 0; i < n; ++i) lens[i] = shards[i].size();
    return ugo_fec_check_shards(n, lens.data(), nilOK ? 1 : 0, S);
  }
  int Encode(std::vector<std::vector<uint8_t>>& shards) {
    size_t S = 0;
    if (int st = check(shards, false, &S)) return st;
    const size_t n = d + p, P = pitch(S);
    uint8_t* buf = staging(n * P);
    for (int k = 0; k < d; ++k) std::memcpy(buf + k * P, shards[k].data(), S);
    if (int st = ugo_fec_encode_host(ctx, buf, 1, S, P)) return st;
    for (size_t k = d; k < n; ++k) std::memcpy(shards[k].data(), buf + k * P, S);
    return UGO_FEC_OK;
  }
  int reconstruct(std::vector<std::vector<uint8_t>>& shards, unsigned flags) {
    size_t S = 0;
    if (int st = check(shards, true, &S)) return st;
    const size_t n = d + p, P = pitch(S);
    uint8_t* buf = staging(n * P);
    uint64_t mask[4] = {0, 0, 0, 0};
    for (size_t r = 0; r < n; ++r)
      if (!shards[r].empty()) {
        mask[r / 64] |= 1ull << (r % 64);
        std::memcpy(buf + r * P, shards[r].data(), S);
      }
    int8_t status = 0;
    if (int st = ugo_fec_reconstruct_host(ctx, buf, mask, 1, S, P, flags, &status)) return st;
    const size_t limit = (flags & UGO_FEC_RECONSTRUCT_DATA_ONLY) ? d : n;
    for (size_t r = 0; r < limit; ++r)
      if (shards[r].empty()) shards[r].assign(buf + r * P, buf + r * P + S);
    return UGO_FEC_OK;
  }
};

}  // namespace

int main(int argc, char** argv) {
  const int reps = argc > 1 ? std::atoi(argv[1]) : 2000;
  std::mt19937 rng(0x5EED);

  // calcECC per call
  {
    ugo_fecconn* f = nullptr;
    check(ugo_fecconn_new(RXLIMIT, D, P, 0, &f), "new");
    std::vector<std::vector<uint8_t>> bufs(N, std::vector<uint8_t>(PKT));
    for (auto& b : bufs)
      for (auto& x : b) x = static_cast<uint8_t>(rng());
    std::vector<uint8_t*> ptrs(N);
    std::vector<size_t> lens(N, PKT);
    for (int k = 0; k < N; ++k) ptrs[k] = bufs[k].data();
    for (int i = 0; i < 200; ++i) check(ugo_fecconn_calc_ecc(f, ptrs.data(), lens.data(), N, 6, PKT), "calc_ecc");
    std::vector<double> t;
    for (int i = 0; i < reps; ++i) {
      const auto t0 = clk::now();
      check(ugo_fecconn_calc_ecc(f, ptrs.data(), lens.data(), N, 6, PKT), "calc_ecc");
      t.push_back(us_since(t0));
    }
    report("calc_ecc", t, "us per call (one group)");
    check(ugo_fecconn_service(f, 0), "service");
    for (int i = 0; i < 200; ++i) check(ugo_fecconn_calc_ecc(f, ptrs.data(), lens.data(), N, 6, PKT), "calc_ecc");
    t.clear();
    for (int i = 0; i < reps; ++i) {
      const auto t0 = clk::now();
      check(ugo_fecconn_calc_ecc(f, ptrs.data(), lens.data(), N, 6, PKT), "calc_ecc");
      t.push_back(us_since(t0));
    }
    report("svc_calc_ecc", t, "us per call (one group)");
    ugo_fecconn_free(f);
  }

  // Encoder.Encode at G = 1 on a pinned group
  {
    ugo_fec* ctx = nullptr;
    check(ugo_fec_create(0, D, P, &ctx), "create");
    void* p = nullptr;
    const size_t S = PKT - 6, pitch = (S + 15) / 16 * 16;
    check(ugo_fec_host_alloc(N * pitch, &p), "host_alloc");
    auto* g = static_cast<uint8_t*>(p);
    for (size_t i = 0; i < N * pitch; ++i) g[i] = static_cast<uint8_t>(rng());
    for (int i = 0; i < 200; ++i) check(ugo_fec_encode_host(ctx, g, 1, S, pitch), "encode_host");
    std::vector<double> t;
    for (int i = 0; i < reps; ++i) {
      const auto t0 = clk::now();
      check(ugo_fec_encode_host(ctx, g, 1, S, pitch), "encode_host");
      t.push_back(us_since(t0));
    }
    report("encode_host_g1", t, "us per call (one group)");
    ugo_fec_host_free(p);
    ugo_fec_destroy(ctx);
  }

  // the cgo shim's call sequence
  {
    GoShim shim;
    shim.d = D;
    shim.p = P;
    check(ugo_fec_create(0, D, P, &shim.ctx), "create");
    auto group = [&](size_t S) {
      std::vector<std::vector<uint8_t>> g(N, std::vector<uint8_t>(S));
      for (auto& b : g)
        for (auto& x : b) x = static_cast<uint8_t>(rng());
      return g;
    };
    auto time_case = [&](const char* name, size_t S, auto&& call) {
      auto g = group(S);
      check(shim.Encode(g), "shim encode");
      for (int i = 0; i < 200; ++i) call(g);
      std::vector<double> t;
      for (int i = 0; i < reps; ++i) {
        const auto t0 = clk::now();
        call(g);
        t.push_back(us_since(t0));
      }
      report(name, t, "us per call (one group)");
    };
    // then the same calls with the per-call service on (ugo_fec_service_start:
    // a resident workgroup serves them, no launch and no synchronize per call)
    for (int svc = 0; svc < 2; ++svc) {
      if (svc) check(ugo_fec_service_start(shim.ctx, 0), "service_start");
      const std::string pre = svc ? "svc_shim_" : "shim_";
      time_case((pre + "encode_1470").c_str(), PKT - 6, [&](auto& g) { check(shim.Encode(g), "shim encode"); });
      time_case((pre + "reconstruct_1476_1loss").c_str(), PKT, [&](auto& g) {
        auto w = g;
        w[3].clear();
        check(shim.reconstruct(w, 0), "shim reconstruct");
      });
      time_case((pre + "reconstruct_data_1476_1loss").c_str(), PKT, [&](auto& g) {
        auto w = g;
        w[3].clear();
        check(shim.reconstruct(w, UGO_FEC_RECONSTRUCT_DATA_ONLY), "shim reconstruct data");
      });
    }
    check(ugo_fec_service_stop(shim.ctx), "service_stop");
    if (shim.stage) ugo_fec_host_free(shim.stage);
    ugo_fec_destroy(shim.ctx);
  }

  // input: lossless / lossy per call / lossy batched
  std::vector<uint8_t> out(size_t(4096) * D * PKT);
  auto run = [&](const char* name, int drop, int batch, unsigned flags = 0, bool svc = false) {
    const int gpr = std::max(64, batch);  // groups per repetition
    const int nrep = std::max(10, reps / gpr);
    ugo_fecconn* f = nullptr;
    check(ugo_fecconn_new(RXLIMIT, D, P, 0, &f), "new");
    if (svc) check(ugo_fecconn_service(f, 0), "service");
    int nrec = 0;
    size_t rl = 0;
    check(ugo_fecconn_set_batch_ex(f, batch, flags, out.data(), out.size(), &nrec, &rl), "set_batch");
    uint32_t base = 0;
    std::vector<double> t;
    long recovered = 0;
    // batched: one continuous stream, flushed once at its end (a flush per
    // repetition would wait for every batch the moment it is launched);
    // per call: repetitions timed one by one
    std::vector<std::vector<std::vector<uint8_t>>> reps_pk;
    for (int r = 0; r < nrep + 3; ++r) {
      reps_pk.push_back(stream(base, gpr, drop, rng));
      base += static_cast<uint32_t>(gpr * N);
    }
    double total = 0;
    for (int r = -3; r < nrep; ++r) {  // 3 untimed repetitions
      const auto& pk = reps_pk[r + 3];
      const auto t0 = clk::now();
      for (const auto& w : pk) {
        uint32_t seq;
        uint16_t flag;
        check(ugo_fecconn_input(f, w.data(), w.size(), &seq, &flag, out.data(), out.size(), &nrec, &rl), "input");
        recovered += nrec;
      }
      if (batch == 0 || r == -1 || r == nrep - 1) {
        check(ugo_fecconn_flush(f, out.data(), out.size(), &nrec, &rl), "flush");
        recovered += nrec;
      }
      const double us = us_since(t0);
      if (r >= 0) {
        t.push_back(us / gpr);
        total += us;
      }
    }
    const long want = drop >= 0 && drop < D ? static_cast<long>(nrep + 3) * gpr : 0;
    if (recovered != want) {
      std::fprintf(stderr, "%s: recovered %ld shards, expected %ld\n", name, recovered, want);
      std::exit(1);
    }
    report(name, t, batch ? "us per group (all its input calls; repetitions of one stream, the last one "
                            "with the final flush)" : "us per group (all its input calls)", gpr,
           total / (double(nrep) * gpr));
    ugo_fecconn_free(f);
  };
  run("input_lossless", -1, 0);
  run("input_lossy", 3, 0);
  run("svc_input_lossy", 3, 0, 0, true);
  run("input_batch_16", 3, 16);
  run("input_batch_64", 3, 64);
  run("input_batch_256", 3, 256);
  run("input_batch_16_overlap", 3, 16, UGO_FECCONN_BATCH_OVERLAP);
  run("input_batch_64_overlap", 3, 64, UGO_FECCONN_BATCH_OVERLAP);
  run("input_batch_256_overlap", 3, 256, UGO_FECCONN_BATCH_OVERLAP);
  return 0;
}
