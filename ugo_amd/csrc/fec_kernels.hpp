// fec_kernels.hpp -- internal interface between the C-ABI (ugo_fec.cpp) and
// the gfx950 kernels (fec_kernels.hip).  Not part of the public ABI.
#pragma once
#include <hip/hip_runtime_api.h>

#include <cstdint>

namespace ugo {
namespace kern {

// One launch covers groups [g0, g0 + items / chunks) of the batch.
struct Batch {
  uint8_t* base;            // row r of group g at base + g*gstride + r*rstride (device)
  const uint8_t* desc;      // descriptor (MODE 0), table (MODE 1), workspace (MODE 2)
  const uint64_t* present;  // device presence masks (MODE 1/2)
  int8_t* status;           // device per-group status, nullable
  uint64_t g0;              // first group of this launch
  uint64_t g_desc0;         // group whose descriptor sits at desc (MODE 2)
  uint64_t gstride;         // bytes between consecutive groups
  uint64_t rstride;         // bytes between consecutive rows of one group
  uint64_t nmask;           // (1 << (d+p)) - 1
  uint32_t S;               // shard size in bytes
  uint32_t chunks;          // column chunks per group (16 B, or 4 B for the byte kernel)
  uint32_t items;           // groups_in_launch * chunks
  uint32_t desc_stride;
  uint32_t d;
  uint32_t dpad;
  uint32_t epad;
  uint32_t data_only;
  uint32_t pass;            // k_apply_w with CPT > 1: item distance between a thread's chunks
  const uint32_t* mult;     // gf::perm_tables (256 x 8 dwords, device) for k_apply_p
  uint8_t* out;             // reconstruct: null = erased rows rebuilt in place; else output i
  uint64_t ogstride;        //   (i-th erased row, ascending) of group g at out + g*ogstride + i*orstride
  uint64_t orstride;
  const uint64_t* rows;     // k_apply_rows: row r of group g at rows[g*n + r] (device addresses)
  uint32_t n;               // k_apply_rows: d + p; k_apply_pd: groups in the launch
  const uint32_t* list;     // list form (launch_apply_list): entry j = g0 + gl reads group list[j]'s rows
  const uint32_t* count;    //   and writes output / status j; entries at or past *count do nothing
  const uint32_t* rowoff;   // list form, nullable: entry j's output i is row rowoff[j] + i of out (row-compact,
  uint32_t* rowid;          //   out + row*orstride), and rowid[rowoff[j] + i] = list[j]*n + its erased row
                            //   (nullable; needs rowoff; n = d + p)
  uint32_t max_rows;        //   with rowoff: rows at or past max_rows are not written
};

struct Prep {
  uint8_t* desc;            // workspace: one descriptor per group
  const uint64_t* present;
  const uint8_t* M;         // (d+p) x d encoding matrix (device)
  const uint8_t* gf_exp;    // 512 B
  const uint8_t* gf_log;    // 256 B
  uint64_t g0;
  uint64_t g_desc0;
  uint64_t nmask;
  uint32_t desc_stride;
  uint32_t d;
  uint32_t n;
  uint32_t dpad;
  uint32_t epad;
};

int apply_dmax(int d);  // register-array bucket for k_apply, 0 if d > 32
bool has_const_encode(int d, int p);
hipError_t launch_encode_const(int d, int p, const Batch& a, hipStream_t s);
hipError_t launch_apply(int mode, int dmax, const Batch& a, hipStream_t s);
hipError_t launch_apply_bytes(int mode, const Batch& a, hipStream_t s);
hipError_t launch_prepare(const Prep& a, uint32_t groups, hipStream_t s);
hipError_t launch_apply_rows(int mode, const Batch& a, hipStream_t s);  // MODE 1 / 2, output batch required
// List form of the MODE-1 reconstruct (d + p <= 16): a.items = max entries * chunks;
// entry j reads the rows of group a.list[j] and writes output slot / status j.
hipError_t launch_apply_list(int dmax, const Batch& a, hipStream_t s);
// Lossy-group list: the groups of [0, groups) with an erased row to rebuild
// (data rows only when data_only), ascending, into list[0 .. *count); `work`
// holds 2 * ceil(groups / kLossyPerBlock) words of scratch.  rowoff (nullable):
// rowoff[j] = the rows to rebuild in entries before j, counting only groups
// with >= d present rows (the others rebuild nothing), and *rows (nullable)
// their total: the row-compact output offsets of launch_apply_list.
constexpr uint32_t kLossyPerBlock = 4096;
hipError_t launch_lossy_list(const uint64_t* present, uint64_t groups, uint64_t nmask, uint64_t dmask, uint32_t d,
                             uint32_t* list, uint32_t* count, uint32_t* rowoff, uint32_t* rows, uint32_t* work,
                             hipStream_t s);
// The same in one launch: `words` = one u64 per tile of context-owned memory
// (zeroed once), reused by the calls of one stream with a new `epoch` each
// (never 0).
hipError_t launch_lossy_list1(const uint64_t* present, uint64_t groups, uint64_t nmask, uint64_t dmask, uint32_t d,
                              uint32_t* list, uint32_t* count, uint32_t* rowoff, uint32_t* rows, uint64_t* words,
                              uint32_t epoch, hipStream_t s);
// Dense rows (group stride == S, no padding; k_apply_pd): MODE 1 / 2, d <= 16
// (dmax 4..16), p <= 4, S >= kDenseMinS (a wave's 63 chunks span at most one
// group boundary).  a.base = row 0 of group a.g0, 16-B aligned; a.items =
// ceil(groups * S / 16); a.n = groups in the launch.
constexpr uint32_t kDenseMinS = 63 * 16 + 1;
hipError_t launch_apply_dense(int mode, int dmax, const Batch& a, hipStream_t s);


// Per-call service (ugo_fec_service_*): one resident block polls a mailbox in
// pinned host memory and runs each small group-major host batch it is handed
// (zero-copy, through the descriptor path), so a per-group call costs neither
// a launch nor a stream synchronize.  Protocol: the host fills the request,
// then bumps seq; the block serves it, then stores done = seq.  The block
// leaves after idle_ticks (wall clock) without a request or on kSvcStop, and
// clears `alive` as its last store; the host relaunches on its next request.
constexpr int kSvcMaxGroups = 16;
struct SvcBox {
  // request line (host -> device): four 16-B pieces, each {tag, 3 words};
  // the host writes every field, then the tags, then piece 0's tag (seq).
  // The poll reads the whole line in one load and takes it when all four tags
  // equal a new seq (a 16-B piece is read whole):
  //   [0] seq  [1] op        [2] groups     [3] S
  //   [4] tag  [5] shards lo [6] shards hi  [7] flags
  //   [8] tag  [9] pitch lo  [10] pitch hi  [11] present[0] lo
  //   [12] tag [13] present[0] hi [14] present[1] lo [15] present[1] hi
  alignas(64) uint32_t line[16];
  alignas(64) uint64_t present[kSvcMaxGroups];  // reconstruct: masks of groups 2 and up
  alignas(64) uint32_t done;                     // device -> host
  uint32_t alive;
  int8_t status[kSvcMaxGroups];
#ifdef UGO_SVC_TRACE  // A/B builds only (tools/svc_trace.cpp): wall-clock ticks of a request's phases
  alignas(64) uint64_t trace[8];
#endif
};
enum : uint32_t { kSvcEncode = 1, kSvcReconstruct = 2, kSvcStop = 3 };
struct SvcArgs {
  Batch a;                  // d, dpad, epad, desc_stride, nmask, mult; a.desc = MODE-1 table
  const uint8_t* encdesc;   // encode descriptor (MODE 0)
  SvcBox* box;              // device view of the mailbox
  uint64_t idle_ticks;
  uint32_t start_seq;       // the last seq on the line that must not be served (served, or abandoned)
  uint64_t stall_ticks;     // tests only (ugo_fec_service_config): wait this long before serving each request
};
// dmax 4..16 (d <= 16) and p <= 4 (epad 4) only
hipError_t launch_service(int dmax, const SvcArgs& sa, hipStream_t s);

}  // namespace kern
}  // namespace ugo
