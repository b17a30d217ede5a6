// svc_trace.cpp -- where a served per-group call's time goes.  Needs a library
// built with -DUGO_SVC_TRACE (tools/build_variant.sh svctrace -DUGO_SVC_TRACE),
// whose k_service records wall-clock ticks (100 MHz) per request:
//   t0 request seen (after the poll's acquire)   t1 request decoded (block barrier)
//   t2 wave 0's row loads landed                 t3 wave 0's stores issued
//   t4 wave 0's stores drained (vmcnt 0)         t5 every wave drained (barrier)
// and the host times each call.  Prints medians.  Not product code.
// Build: g++ -O2 -std=c++17 -o tools/svc_trace tools/svc_trace.cpp -Lbuild_ab/svctrace -lugofec -Wl,-rpath,'$ORIGIN/../build_ab/svctrace'
#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#include "../include/ugo_fec.h"

extern "C" int ugo_fec_svc_trace(const ugo_fec* c, uint64_t* out);

static double med(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? std::atoi(argv[1]) : 3000;
  const int d = 10, p = 3, n = 13;
  const size_t S = 1470, pitch = 1472;
  ugo_fec* c = nullptr;
  if (ugo_fec_create(0, d, p, &c)) return 1;
  uint8_t* buf = nullptr;
  if (ugo_fec_host_alloc(n * pitch, reinterpret_cast<void**>(&buf))) return 1;
  std::memset(buf, 7, n * pitch);
  if (ugo_fec_service_start(c, 1000000)) return 1;
  for (int i = 0; i < 200; ++i)
    if (ugo_fec_encode_host(c, buf, 1, S, pitch)) return 1;
  std::vector<double> host, ph[5], total;
  for (int i = 0; i < reps; ++i) {
    const auto t0 = std::chrono::steady_clock::now();
    if (ugo_fec_encode_host(c, buf, 1, S, pitch)) return 1;
    host.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    uint64_t t[6];
    if (ugo_fec_svc_trace(c, t)) return 1;
    for (int k = 0; k < 5; ++k) ph[k].push_back((t[k + 1] - t[k]) / 100.0);  // 100 MHz ticks -> us
    total.push_back((t[5] - t[0]) / 100.0);
  }
  std::printf("{\"host_call_us\": %.3f, \"device_t0_t5_us\": %.3f, \"decode_us\": %.3f, \"row_loads_us\": %.3f, "
              "\"compute_issue_us\": %.3f, \"store_drain_us\": %.3f, \"barrier_us\": %.3f, \"reps\": %d}\n",
              med(host), med(total), med(ph[0]), med(ph[1]), med(ph[2]), med(ph[3]), med(ph[4]), reps);
  ugo_fec_service_stop(c);
  ugo_fec_host_free(buf);
  ugo_fec_destroy(c);
  return 0;
}
