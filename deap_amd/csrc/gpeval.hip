// gpeval.hip — MI355X (gfx950) GP population evaluator: HIP kernels + C ABI.
//
// Replaces the reference's per-individual hot path
//     toolbox.map(toolbox.evaluate, invalid_ind)       deap/algorithms.py:172
//       -> gp.compile(individual, pset)                 deap/gp.py:462-487
//       -> per-case Python loop + math.fsum / sum       examples/gp/*.py
// by one batched evaluation of a whole generation of flattened programs
// (deap_amd/flatten.py) over fitness cases resident in HBM.
//
// One translation unit; besides the generated cores (gp_asm_*.inc) its parts
// are: trig_dev.h (sin/cos; glibc restated), exact_int.h (Python's exact
// ints on the device and the host), rccl_layer.h (case sharding's combine
// kernels, RCCL via dlopen), select_dev.h (device lexicase / tournament),
// ctx.h (the context and launch plans), fb_kernels.h (the C++ F and B
// interpreters), asm_kernels.h (the kernels around the generated cores),
// planner.h (launch geometry, plan(), the launches), exact_run.h (the
// glibc-exact and exact-int passes); this file holds the device lowering,
// the threaded-code translation, the run paths and the C ABI.
//
// Execution model:
//   * one wavefront interprets one program at a time; its 64 lanes hold
//     64*K fitness cases (K per lane).  The program is wave-uniform, so
//     instruction words are fetched with scalar loads and dispatched with
//     scalar branches; the per-case arithmetic is plain VALU.
//   * the F machine keeps the accumulator T (K doubles) in VGPRs and the
//     rarely used operand stack (Sethi-Ullman ordering keeps it <= 5 deep) in
//     LDS; the B machine does the same with 32-case bit-planes.
//   * a workgroup (4 waves) stages one tile of cases (all variables, 64*K
//     cases) into LDS and its waves run their P programs each over that tile
//     before the next tile is staged, so each case is read from HBM once per
//     program group and the program stream comes from the scalar cache.
//   * per (program, tile): lane partials -> wave reduction -> lane j of the
//     wave accumulates program j across the tiles of its tile group; one
//     partial per (tile group, program) goes to HBM and a second kernel sums
//     the tile groups in fixed order (deterministic).
//   * MSE is accumulated as a double-double (TwoSum), so the final
//     fl(hi + lo) is the correctly rounded sum of the per-case terms, i.e.
//     what math.fsum returns (symbreg.py:61), barring ties at 2^-106.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <array>

#include "host_pool.h"
#include <rccl/rccl.h>   // types only: RCCL is opened with dlopen
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <string>
#include <thread>
#include <type_traits>
#include <vector>

#include "../../include/gpeval.h"
#include "lower_core.h"
#include "gp_asm_core.inc"
#include "gp_asm_core32.inc"
#include "gp_asm_core_deep.inc"
#include "gp_asm_core32_deep.inc"
#include "gp_asm_layout.h"
#include "gp_asm_layout_deep.h"
#include "gp_asm_core_exact.inc"
#include "gp_asm_layout_exact.h"
#include "gp_asm_core_typed.inc"
#include "gp_asm_layout_typed.h"
#include "gp_asm_core_exact_deep.inc"
#include "gp_asm_layout_exact_deep.h"


namespace {

// Opcodes — keep in sync with deap_amd/flatten.py:Op.
enum : uint32_t {
  OP_END = 0, OP_LDV = 1, OP_LDC = 2, OP_PUSH = 3, OP_PUSHV = 4, OP_PUSHC = 5,
  OP_ADD = 8, OP_SUB = 11, OP_RSUB = 14, OP_MUL = 17, OP_DIV = 20,
  OP_RDIV = 23, OP_LT = 26, OP_GT = 29, OP_EQ = 32, OP_AND = 35, OP_OR = 38,
  OP_XOR = 41, OP_NEG = 48, OP_SIN = 49, OP_COS = 50, OP_NOT = 51,
  OP_ITE = 52, OP_NPDIV = 56, OP_RNPDIV = 59
};

constexpr int kWaves = 4;
constexpr int kBlock = 64 * kWaves;
constexpr int kFMaxBlock = 512;     // f_eval: 4 or 8 waves per block
// f_eval_asm: 4, 8 or 16 waves/block; a core past 112 VGPRs (more cases
// per lane) cannot run 4 waves per SIMD, so its blocks stay at 8 waves
constexpr int kAsmMaxBlock = asmcore::VGPRS > 140 ? 512 : asmcore::VGPRS > 112 ? 768 : 1024;
constexpr int kAsmDeepMaxBlock = 512;  // ... deep cores: 4 or 8 (>128 VGPRs)
constexpr int kFastDepth = 6;     // operand-stack slots of the fast kernels
constexpr int kDeepDepth = 32;    // ... of the fallback kernels
constexpr int kFK = 2;            // cases per lane, F machine fast kernel
constexpr uint32_t kRedoListCap = 1u << 22;   // (program, tile) pairs
constexpr int kFK32 = 4;          // ... in fp32 mode (same LDS bytes as kFK)

struct Task {
  const uint32_t* code;
  const int64_t* off;
  const int32_t* slot_prog;  // slot -> program (or -1)
  int64_t n_slots;
  int P;                     // programs per wave
  const void* X;             // F: double[nv][n]; B: uint32[nv][n_words]
  int nv;
  const void* terms;         // F: double[nt][n]; B: uint32[n_words]
  int nt;
  int64_t n_cases;           // F: cases; B: bits
  int64_t n_units;           // F: cases; B: words
  int64_t n_tiles;
  int tiles_per_group;
  double* part;              // [group][slot][2]
  double* case_out;          // optional [program][n_cases] per-case terms
  unsigned long long* first_err;  // [program]
  uint32_t* flags;                // [program]
  int sdepth;                     // f_eval: LDS stack slots per wave (<= D)
  int gtab_lds;                   // EXACT f_eval: glibc's tables copied to LDS
};

__host__ __device__ __forceinline__ double dbits(uint32_t lo, uint32_t hi) {
  const uint64_t v = (uint64_t)lo | ((uint64_t)hi << 32);
  double d;
  __builtin_memcpy(&d, &v, 8);
  return d;
}

// Program words of the C++ interpreters: the first 64 words are loaded once
// into one VGPR (lane i holds word i) and read with v_readlane; later words
// come from memory.  The device code buffer carries kCodePad END words past
// the last program, so lanes beyond a program's end read valid memory.
constexpr int kCodePad = 64;
struct ProgWords {
  const uint32_t* pc0;
  uint32_t win;
  __device__ __forceinline__ ProgWords(const uint32_t* pc, int lane)
      : pc0(pc), win(pc[lane]) {}
  // with the window already loaded (f_eval prefetches the next program's)
  __device__ __forceinline__ ProgWords(const uint32_t* pc, uint32_t w)
      : pc0(pc), win(w) {}
  __device__ __forceinline__ uint32_t operator[](uint32_t i) const {
    return i < 64u ? (uint32_t)__builtin_amdgcn_readlane((int)win, (int)i)
                   : pc0[i];
  }
};

// TwoSum with non-finite guard: keeps inf/nan in hi, lo = 0.
__device__ __forceinline__ void two_sum(double a, double b, double& s,
                                        double& e) {
  s = a + b;
  double bb = s - a;
  e = (a - (s - bb)) + (b - bb);
  if (!__builtin_isfinite(s)) e = 0.0;
}

__device__ __forceinline__ void dd_add(double& hi, double& lo, double bhi,
                                       double blo) {
  double s, e;
  two_sum(hi, bhi, s, e);
  e = e + (lo + blo);
  double h = s + e;
  double l = e - (h - s);
  if (!__builtin_isfinite(h)) l = 0.0;
  hi = h;
  lo = l;
}

__device__ __forceinline__ int uniform(int v) {
  return __builtin_amdgcn_readfirstlane(v);
}

__device__ __forceinline__ double shfl_xor_d(double v, int m) {
  return __shfl_xor(v, m, 64);
}


}  // namespace
#include "trig_dev.h"
#include "exact_int.h"
#include "fb_kernels.h"
#include "asm_kernels.h"
#include "rccl_layer.h"
namespace {

// ------------------------------------------------- device lowering ----
// The host flattener's lowering (lower_core.h, the same source) run on the
// device, one thread per tree: the host only maps node objects to entry
// codes (one byte per node, prefix order; 255 = the tree's next ephemeral
// value) and uploads them; records, folds and words are made here.
struct DevTrig {   // folded sin/cos constants: glibc's algorithm (= libm)
  __host__ __device__ static double sin(double x) { return glibc_trig(x, false); }
  __host__ __device__ static double cos(double x) { return glibc_trig(x, true); }
};
struct CodeEnts {  // reversed-prefix view of one tree's codes
  const uint8_t* c;
  int64_t len;
  int32_t eph;     // the tree's ephemerals are numbered in prefix order
  __device__ int32_t operator()(int64_t k) {
    const uint8_t v = c[len - 1 - k];
    return v != 255 ? (int32_t)v : -1 - (eph--);
  }
};
static_assert(sizeof(lowering::Val) == sizeof(gpe_value) &&
                  sizeof(lowering::Entry) == sizeof(gpe_entry),
              "gpe_value / gpe_entry are lowering::Val / Entry");

// IL: interleaved scratch — the trees of one wave share a region of rows
// (wrow[w] .. wrow[w + 1]: the wave's longest tree) and record k of lane l's
// tree sits at (wrow[w] + k)·64 + l, its words at (wword[w] + j)·64 + l: the
// lanes' accesses to one node index are adjacent (the build pass's are all
// to the same index).  Otherwise each tree's scratch is contiguous.
template <bool IL>
__global__ __launch_bounds__(128) void lower_trees(
    const uint8_t* codes, const int64_t* node_off, const int64_t* eph_off,
    const lowering::Val* evals, lowering::Tables T, int64_t n, lowering::PRec* rec,
    int32_t* stk, lowering::Val* cv, double* ib, uint32_t* words, const int64_t* wrow,
    const int64_t* wword, uint32_t* n_words, uint32_t* meta) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t base = node_off[i], len = node_off[i + 1] - base;
  CodeEnts E{codes + base, len, (int32_t)(eph_off[i + 1] - eph_off[i] - 1)};
  lowering::Result r;
  constexpr int S = IL ? 64 : 1;
  const int64_t eb = IL ? wrow[i >> 6] * 64 + (i & 63) : base;
  lowering::Strided<uint32_t, S> out{IL ? words + wword[i >> 6] * 64 + (i & 63)
                                        : words + 3 * base + i};
  lowering::lower<DevTrig>(T, E, len, evals + eph_off[i], lowering::PackedRecsS<S>{rec + eb},
                           lowering::Strided<int32_t, S>{stk + eb},
                           lowering::Strided<lowering::Val, S>{cv + eb},
                           lowering::Strided<double, S>{ib ? ib + eb : nullptr}, out, r);
  // what validate_program reports for trusted words: asm-capable, and the
  // planner's cost inputs — sin/cos and protectedDiv counts (meta bits 15-26
  // and 27-31, clamped: a cost estimate only, the planner's order and not
  // any value depends on it)
  const bool F = T.machine == 0;
  bool ok = F && r.depth <= asmcore_deep::D;
  uint32_t n_trig = 0, n_div = 0;
  for (int32_t j = 0; j < r.n_words; ++j) {
    const uint32_t w = out[j];
    const uint32_t op = w & 0xffu, x = w >> 16;
    if (op == OP_END) break;
    bool konst = op == OP_LDC || op == OP_PUSHC, var = op == OP_LDV || op == OP_PUSHV;
    if ((op >= OP_ADD && op < OP_NEG) || (op >= OP_NPDIV && op < OP_NPDIV + 6)) {
      const bool np = op >= OP_NPDIV;
      const uint32_t fam = np ? 12 + (op - OP_NPDIV) / 3 : (op - OP_ADD) / 3;
      const uint32_t form = np ? (op - OP_NPDIV) % 3 : (op - OP_ADD) % 3;
      if (fam > 5 && !np) ok = false;
      n_div += np || fam == 4 || fam == 5;
      var = form == 1;
      konst = form == 2;
    } else if (op == OP_SIN || op == OP_COS) {
      ++n_trig;
    } else if (op == OP_NOT || op == OP_ITE) {
      ok = false;
    }
    if (var && (int)x >= asmcore::NV) ok = false;
    if (konst && F) j += 2;
  }
  n_words[i] = (uint32_t)r.n_words;
  meta[i] = (uint32_t)min(r.depth, 255) | ((uint32_t)r.err << 8) |
            ((uint32_t)r.declined << 11) | ((uint32_t)r.inexact << 12) |
            ((uint32_t)r.verr << 13) | ((uint32_t)ok << 14) |
            (min(n_trig, 0xfffu) << 15) | (min(n_div, 31u) << 27);
}
template <bool IL>
__global__ void compact_words(const uint32_t* words, const int64_t* node_off,
                              const int64_t* wword, const int64_t* off, int64_t n,
                              uint32_t* code) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  constexpr int S = IL ? 64 : 1;
  const uint32_t* src =
      IL ? words + wword[i >> 6] * 64 + (i & 63) : words + 3 * node_off[i] + i;
  for (int64_t j = off[i], k = 0; j < off[i + 1]; ++j, ++k) code[j] = src[k * S];
}
// the OP_END pad after the last program (its start is only known on the device)
__global__ void pad_code(uint32_t* code, const int64_t* off, int64_t n, int pad) {
  const int j = threadIdx.x;
  if (j < pad) code[off[n] + j] = 0u;
}
struct U32ToI64 {
  __host__ __device__ int64_t operator()(uint32_t x) const { return (int64_t)x; }
};
struct U16ToI64 {
  __host__ __device__ int64_t operator()(uint16_t x) const { return (int64_t)x; }
};

}  // namespace
#include "select_dev.h"

#include "ctx.h"

namespace {

int fail(gpe_ctx* c, int code, const std::string& msg) {
  if (c) c->err = msg;
  return code;
}

// Waiting on a stream that holds RCCL collectives: a rank that never joins
// (a crashed peer, a mismatched call sequence) would block
// hipStreamSynchronize forever, leaving the job to the launcher's own limit
// with no diagnosis.  The wait polls instead, at most comm_timeout_s()
// seconds (GPE_COMM_TIMEOUT_S, default 120); query() returns 0 when the
// stream is done, 1 while busy, -1 on an error.
double comm_timeout_s() {
  const char* e = getenv("GPE_COMM_TIMEOUT_S");
  const double v = e ? atof(e) : 0.0;
  return v > 0.0 ? v : 120.0;
}
template <typename Q>
int bounded_wait(double timeout_s, Q query) {
  const auto t0 = std::chrono::steady_clock::now();
  for (int spin = 0;; ++spin) {
    const int q = query();
    if (q <= 0) return q == 0 ? 0 : GPE_E_HIP;
    if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() >
        timeout_s)
      return GPE_E_COMM;
    if (spin > 64) std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
}
std::string comm_timeout_msg(const char* what, int rank, int world, double timeout_s,
                             const char* async_error) {
  char buf[256];
  snprintf(buf, sizeof(buf),
           "%s: collective not complete after %.0f s on rank %d of %d (RCCL async "
           "error: %s); communicator aborted",
           what, timeout_s, rank, world, async_error);
  return buf;
}
// The context stream after a collective, bounded; on expiry the
// communicator is asked for its asynchronous error and aborted (its pending
// collectives then drain), and the call fails with GPE_E_COMM.
int comm_sync(gpe_ctx* ctx, const char* what) {
  const double limit = comm_timeout_s();
  hipError_t last = hipSuccess;
  const int rc = bounded_wait(limit, [&]() {
    last = hipStreamQuery(ctx->stream);
    return last == hipSuccess ? 0 : last == hipErrorNotReady ? 1 : -1;
  });
  if (rc == GPE_E_HIP)
    return fail(ctx, GPE_E_HIP, std::string(what) + ": " + hipGetErrorString(last));
  if (rc == GPE_E_COMM) {
    RcclApi& r = rccl();
    ncclResult_t ae = ncclSuccess;
    if (ctx->comm && r.async_error) (void)r.async_error(ctx->comm, &ae);
    const std::string msg = comm_timeout_msg(what, ctx->comm_rank, ctx->comm_world, limit,
                                             r.error_string ? r.error_string(ae) : "?");
    if (ctx->comm && r.comm_abort) (void)r.comm_abort(ctx->comm);
    ctx->comm = nullptr;
    // the timing events bracket an aborted collective: nothing to report;
    // later sharded calls fail with "communicator aborted" (comm_aborted)
    ctx->comm_timed = ctx->redo_timed = false;
    ctx->comm_aborted = true;
    return fail(ctx, GPE_E_COMM, msg);
  }
  return 0;
}


#define HIPCHK(call)                                                      \
  do {                                                                    \
    hipError_t e_ = (call);                                               \
    if (e_ != hipSuccess)                                                 \
      return fail(ctx, GPE_E_HIP, std::string(#call ": ") +               \
                                      hipGetErrorString(e_));             \
  } while (0)

int host_threads() { return hostpool::threads(); }

// GPE_DIAG lines: a steady-clock stamp in ms (mod 10^5 s), to line up the
// laps of different calls and threads
double diag_stamp() {
  const double ms = std::chrono::duration<double, std::milli>(
                        std::chrono::steady_clock::now().time_since_epoch()).count();
  return ms - 1e8 * (double)(int64_t)(ms / 1e8);
}

// ctx->h_pin with at least `bytes` (grown, never shrunk); nullptr on failure
char* pinned_buf(char** buf, size_t* cap, size_t bytes) {
  if (bytes <= *cap && *buf) return *buf;
  if (*buf) (void)hipHostFree(*buf);
  *buf = nullptr;
  *cap = 0;
  const size_t want = std::max<size_t>(bytes, (size_t)1 << 20);
  if (hipHostMalloc((void**)buf, want, hipHostMallocDefault) != hipSuccess) return nullptr;
  *cap = want;
  return *buf;
}
char* pinned(gpe_ctx* ctx, size_t bytes) {
  return pinned_buf(&ctx->h_pin, &ctx->h_pin_cap, bytes);
}

int host_threads();

// Host -> device copies of caller buffers through pinned staging (copied in
// by host threads, then asynchronous copies on ctx->stream; the caller syncs
// before the staging is reused).  Pageable copies of buffers that Python frees
// right after let the runtime pin them in place, and the next stream
// operation then stalled 10-30 ms on the box at pop 1M.
struct HostPiece {
  void* dst;                   // device
  const void* src;             // host
  size_t bytes;
};
int h2d_staged(gpe_ctx* ctx, const HostPiece* pc, int n_pc);

template <typename T>
int ensure(gpe_ctx* ctx, T** ptr, size_t* cap, size_t n) {
  if (n <= *cap && *ptr) return 0;
  if (*ptr) HIPCHK(hipFree(*ptr));
  *ptr = nullptr;
  size_t want = std::max<size_t>(n, 1);
  HIPCHK(hipMalloc((void**)ptr, want * sizeof(T)));
  *cap = want;
  return 0;
}

int h2d_staged_buf(gpe_ctx* ctx, char** buf, size_t* cap, const HostPiece* pc, int n_pc,
                   hipStream_t stream = nullptr);
int h2d_staged(gpe_ctx* ctx, const HostPiece* pc, int n_pc) {
  return h2d_staged_buf(ctx, &ctx->h_pin_in, &ctx->h_pin_in_cap, pc, n_pc);
}
// ... through the pinned buffer *buf (grown as needed), on `stream`
// (nullptr: the context's)
int h2d_staged_buf(gpe_ctx* ctx, char** buf, size_t* cap, const HostPiece* pc, int n_pc,
                   hipStream_t stream) {
  if (!stream) stream = ctx->stream;
  std::vector<size_t> at((size_t)n_pc);
  size_t total = 0;
  for (int k = 0; k < n_pc; ++k) {
    at[(size_t)k] = total;
    total += (pc[k].bytes + 63) / 64 * 64;
  }
  if (!total) return 0;
  char* stage = pinned_buf(buf, cap, total);
  if (!stage) return fail(ctx, GPE_E_HIP, "hipHostMalloc (staging)");
  const int nth = total >= ((size_t)1 << 20) ? host_threads() : 1;
  auto copy = [&](int t) {
    for (int k = 0; k < n_pc; ++k) {
      const size_t a = pc[k].bytes * t / nth, b = pc[k].bytes * (t + 1) / nth;
      if (b > a) std::memcpy(stage + at[(size_t)k] + a, (const char*)pc[k].src + a, b - a);
    }
  };
  if (nth == 1) {
    copy(0);
  } else {
    hostpool::par_run(nth, copy);
  }
  for (int k = 0; k < n_pc; ++k)
    if (pc[k].bytes)
      HIPCHK(hipMemcpyAsync(pc[k].dst, stage + at[(size_t)k], pc[k].bytes,
                            hipMemcpyHostToDevice, stream));
  return 0;
}

// Reject anything the kernels could mis-execute: unknown opcodes, stack
// slots beyond the declared depth, variables beyond the tile, truncated
// constants, a missing END.  Also reports whether the asm core runs it.
std::string validate_program(const uint32_t* w, int64_t n, int machine,
                             int nv, int32_t depth, bool* asm_ok,
                             int64_t* n_trig = nullptr, int64_t* n_div = nullptr) {
  if (depth < 0) return "negative depth";
  if (n_trig) *n_trig = 0;
  if (n_div) *n_div = 0;
  const bool F = machine == GPE_MACHINE_F;
  bool ok = F && depth <= asmcore_deep::D;
  int64_t i = 0;
  while (i < n) {
    const uint32_t op = w[i] & 0xffu, d = (w[i] >> 8) & 0xffu, x = w[i] >> 16;
    ++i;
    if (op == OP_END) {
      *asm_ok = ok;
      return i == n ? std::string() : "words after END";
    }
    bool konst = false, var = false, stack = false, stack2 = false;
    if (op == OP_LDV) var = true;
    else if (op == OP_LDC) konst = true;
    else if (op == OP_PUSH) stack = true;
    else if (op == OP_PUSHV) stack = var = true;
    else if (op == OP_PUSHC) stack = konst = true;
    else if ((op >= OP_ADD && op < OP_NEG) || (op >= OP_NPDIV && op < OP_NPDIV + 6)) {
      const bool np = op >= OP_NPDIV;
      const uint32_t fam = np ? 12 + (op - OP_NPDIV) / 3 : (op - OP_ADD) / 3;
      const uint32_t form = np ? (op - OP_NPDIV) % 3 : (op - OP_ADD) % 3;
      const bool fam_ok = F ? (fam <= 10 || np) : (fam >= 9 && fam <= 11);
      if (!fam_ok) return "opcode " + std::to_string(op) + " not on this machine";
      if (fam > 5 && !np) ok = false;             // comparisons / logic
      if (n_div && (np || fam == 4 || fam == 5)) ++*n_div;
      stack = form == 0;
      var = form == 1;
      konst = form == 2;
    } else if (op == OP_NEG || op == OP_SIN || op == OP_COS) {
      if (!F) return "float opcode on the boolean machine";
      if (op != OP_NEG && n_trig) ++*n_trig;
    } else if (op == OP_NOT) {
      ok = false;
    } else if (op == OP_ITE) {
      stack2 = true;
      ok = false;
    } else {
      return "unknown opcode " + std::to_string(op);
    }
    if (stack && (int32_t)d >= depth) return "stack slot beyond declared depth";
    if (stack2 && (int32_t)d + 1 >= depth) return "stack slot beyond declared depth";
    if (var && (int)x >= nv) return "variable index out of range";
    if (var && (int)x >= asmcore::NV) ok = false;
    static_assert(asmcore_deep::NV == asmcore::NV, "one variable layout");
    if (konst && F) {
      if (i + 2 > n) return "truncated constant";
      i += 2;
    }
  }
  return "missing END";
}

// Flattener words -> threaded code in 16-word windows (handler byte offsets
// + inline constants).  An instruction and the word after it must sit in
// the same window; otherwise a RELOAD word ends the window.  Programs start
// on a window boundary.
// Handler id layout of one core (gp_asm_layout*.h).
struct CoreIds {
  int D, NV, H_END, H_RELOAD, H_LDC, H_LDV0, H_PUSH0, H_PUSHC0, H_PUSHV0, H_BIN0,
      H_FAM_STRIDE, H_NEG, H_SIN, H_COS, H_COUNT;
  int H_NOT = -1, H_ITE0 = -1;      // the typed core only
};
#define CORE_IDS(NS)                                                          \
  CoreIds {                                                                   \
    NS::D, NS::NV, NS::H_END, NS::H_RELOAD, NS::H_LDC, NS::H_LDV0, NS::H_PUSH0, \
        NS::H_PUSHC0, NS::H_PUSHV0, NS::H_BIN0, NS::H_FAM_STRIDE, NS::H_NEG,    \
        NS::H_SIN, NS::H_COS, NS::H_COUNT                                      \
  }
constexpr CoreIds kIds = CORE_IDS(asmcore);
constexpr CoreIds kIdsDeep = CORE_IDS(asmcore_deep);
constexpr CoreIds kIdsExactDeep = CORE_IDS(asmcore_exact_deep);
constexpr CoreIds kIdsTyped = [] {
  CoreIds c = CORE_IDS(asmcore_typed);
  c.H_NOT = asmcore_typed::H_NOT;
  c.H_ITE0 = asmcore_typed::H_ITE0;
  return c;
}();
static_assert(asmcore_typed::WINDOW == asmcore::WINDOW, "one window size");
static_assert(asmcore32::H_COUNT == asmcore::H_COUNT &&
                  asmcore32_deep::H_COUNT == asmcore_deep::H_COUNT &&
                  asmcore32_deep::H_BIN0 == asmcore_deep::H_BIN0 &&
                  asmcore32_deep::H_FAM_STRIDE == asmcore_deep::H_FAM_STRIDE &&
                  asmcore32_deep::H_PUSHV0 == asmcore_deep::H_PUSHV0 &&
                  asmcore32_deep::H_SIN == asmcore_deep::H_SIN &&
                  asmcore32_deep::D == asmcore_deep::D &&
                  asmcore32_deep::K == asmcore32::K &&
                  asmcore_deep::WINDOW == asmcore::WINDOW,
              "the fp32 cores share the fp64 cores' handler layouts and tiles");

// asm core of a program needing `depth` stack slots: 1 = D = 5, 2 = deep
inline uint8_t core_class(bool ok, int32_t depth) {
  return !ok ? 0 : depth <= asmcore::D ? 1 : 2;
}

// Whether the typed core runs a (validated) F-machine program: its families
// (add .. or, opcode order), NEG, NOT, if_then_else, stack slots below
// asmcore_typed::D (if_then_else reads d + 1), at most NV variables; no
// sin/cos, no numpy ops.
HD bool typed_runs(const uint32_t* w) {
  constexpr int D = asmcore_typed::D, NV = asmcore_typed::NV;
  for (;;) {
    const uint32_t op = w[0] & 0xffu, d = (w[0] >> 8) & 0xffu, x = w[0] >> 16;
    ++w;
    if (op == OP_END) return true;
    const bool bin = op >= OP_ADD && op < OP_XOR;      // families 0..10
    const int form = bin ? (int)(op - OP_ADD) % 3 : -1;
    const bool var = op == OP_LDV || op == OP_PUSHV || form == 1;
    const bool konst = op == OP_LDC || op == OP_PUSHC || form == 2;
    const bool slot = op == OP_PUSH || op == OP_PUSHV || op == OP_PUSHC || form == 0;
    if (var && (int)x >= NV) return false;
    if (slot && (int)d >= D) return false;
    if (op == OP_ITE) {
      if ((int)d + 1 >= D) return false;
    } else if (!(bin || op == OP_LDV || op == OP_LDC || op == OP_PUSH || op == OP_PUSHV ||
                 op == OP_PUSHC || op == OP_NEG || op == OP_NOT)) {
      return false;
    }
    if (konst) w += 2;
  }
}

// gpe_set_cases: the cases' NaNs as the default NaN (payload-free; the
// reference's arithmetic never reads a payload)
__global__ __launch_bounds__(256) void canon_nan(double* x, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    if (x[i] != x[i]) x[i] = __builtin_nan("");
}

// HITS_BOOL's constant programs (plan_mode class 5): every case's prediction
// is bool(c), so the hits are the cases whose label has that truth
__global__ __launch_bounds__(256) void const_hits(const uint32_t* kc, int64_t n,
                                                  double t_hits, double f_hits, double* hi,
                                                  double* lo) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t e = kc[i], p = e >> 1;
  hi[p] = (e & 1u) ? t_hits : f_hits;
  lo[p] = 0.0;
}

// One program's threaded code: the handler words of core layout `I` (jump
// words `tab`), inline constants (fp32 core: the constant's fp32 bits), a
// RELOAD word wherever the next instruction would leave its 16-word window
// (END pads the rest); the program starts on a window boundary.  Returns the
// length; writes the words when `out` is not null.  The same code runs on
// the host (gpe_debug_translate, tests) and in translate_kernel.
HD int64_t translate_words(const uint32_t* w, const uint32_t* tab, const CoreIds& I,
                           bool f32, int window_use, uint32_t* out) {
  constexpr int WINDOW = asmcore::WINDOW;
  const int D = I.D, NV = I.NV;
  int64_t n = 0;
  int pos = 0;
  auto emit = [&](uint32_t v) {
    if (out) out[n] = v;
    ++n;
  };
  for (;;) {
    const uint32_t op = w[0] & 0xffu, d = (w[0] >> 8) & 0xffu, x = w[0] >> 16;
    ++w;
    int h;
    bool konst = false;
    if (op == OP_END) {
      emit(tab[I.H_END]);                 // pos <= WINDOW - 1 always holds
      while (n % WINDOW) emit(tab[I.H_END]);
      return n;
    } else if (op == OP_LDV) {
      h = I.H_LDV0 + (int)x;
    } else if (op == OP_LDC) {
      h = I.H_LDC;
      konst = true;
    } else if (op == OP_PUSH) {
      h = I.H_PUSH0 + (int)d;
    } else if (op == OP_PUSHV) {
      h = I.H_PUSHV0 + (int)d * NV + (int)x;
    } else if (op == OP_PUSHC) {
      h = I.H_PUSHC0 + (int)d;
      konst = true;
    } else if (op == OP_NEG) {
      h = I.H_NEG;
    } else if (op == OP_SIN) {
      h = I.H_SIN;
    } else if (op == OP_COS) {
      h = I.H_COS;
    } else if (op == OP_NOT) {
      h = I.H_NOT;
    } else if (op == OP_ITE) {
      h = I.H_ITE0 + (int)d;
    } else {
      // families in handler order: add sub rsub mul div rdiv ndiv nrdiv (the
      // typed core: add .. or, opcode order)
      const bool np = op >= OP_NPDIV;
      const int fam = np ? 6 + (int)(op - OP_NPDIV) / 3 : (int)(op - OP_ADD) / 3;
      const int form = np ? (int)(op - OP_NPDIV) % 3 : (int)(op - OP_ADD) % 3;
      const int base = I.H_BIN0 + fam * I.H_FAM_STRIDE;
      h = form == 0 ? base + (int)d : form == 1 ? base + D + (int)x : base + D + NV;
      konst = form == 2;
    }
    const int need = konst ? 3 : 1;
    if (pos + need > window_use) {            // next word would leave it
      emit(tab[I.H_RELOAD]);
      while (n % WINDOW) emit(tab[I.H_END]);
      pos = 0;
    }
    emit(tab[h]);
    if (konst && f32) {                       // the fp32 core reads fp32 bits
      const double v = __builtin_bit_cast(double, (uint64_t)w[0] | ((uint64_t)w[1] << 32));
      emit(__builtin_bit_cast(uint32_t, (float)v));
      emit(0u);
    } else if (konst) {
      emit(w[0]);
      emit(w[1]);
    }
    if (konst) w += 2;
    pos += need;
  }
}

// words used per window before its RELOAD (GPE_WINDOW_USE: an experiment
// knob pricing the reloads; the full window is WINDOW - 1)
int window_use() {
  static const int v = [] {
    const char* e = getenv("GPE_WINDOW_USE");
    const long u = e ? atol(e) : 0;
    return (int)(u >= 4 && u < asmcore::WINDOW ? u : asmcore::WINDOW - 1);
  }();
  return v;
}

void translate_program(const uint32_t* w, const std::vector<uint32_t>& tab,
                       std::vector<uint32_t>& out, bool f32 = false,
                       const CoreIds& I = kIds) {
  const int64_t n = translate_words(w, tab.data(), I, f32, window_use(), nullptr);
  const size_t base = out.size();
  out.resize(base + (size_t)n);
  translate_words(w, tab.data(), I, f32, window_use(), out.data() + base);
}

// Device translation (translate_device): per program, its core class
// (0: none; 1/2: tab1/I1, tab2/I2; 3: the typed core, decided here by
// typed_runs) -> the length (pass 0) or the words at start[i] (pass 1).
struct XlateTabs {
  const uint32_t* tab[3];
  CoreIds ids[3];
};
__global__ __launch_bounds__(256) void translate_kernel(
    const uint32_t* code, const int64_t* off, const uint8_t* cls, int64_t n,
    XlateTabs T, int f32, int wuse, int pass, uint32_t* len, const uint32_t* start,
    uint32_t* out, uint8_t* typed_ok) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t* w = code + off[i];
  int c = cls ? cls[i] : 0;
  if (typed_ok) {                             // the typed core's programs
    if ((w[0] & 0xffu) == OP_LDC && (w[0] >> 16) == 0 && (w[3] & 0xffu) == OP_END) {
      // one folded constant: its hits need no core run (2: falsy, 3: truthy;
      // bool(nan) is True, as the label test's != 0)
      if (pass == 0) {
        const double v = __hiloint2double((int)w[2], (int)w[1]);
        typed_ok[i] = (uint8_t)(v != 0.0 ? 3 : 2);
        len[i] = 0;
      }
      return;
    }
    c = typed_runs(w) ? 3 : 0;
    if (pass == 0) typed_ok[i] = (uint8_t)(c != 0);
  }
  if (!c) {
    if (pass == 0) len[i] = 0;
    return;
  }
  const int t = c == 3 ? 2 : c - 1;
  if (pass == 0)
    len[i] = (uint32_t)translate_words(w, T.tab[t], T.ids[t], f32 != 0, wuse, nullptr);
  else
    translate_words(w, T.tab[t], T.ids[t], f32 != 0, wuse, out + start[i]);
}

// Threaded code of programs (classes `cls` on the host: 1/2 for the two
// tables given; typed: the typed core decides) into (d_out, d_start), from
// the words already on the device: no host copy of the programs.
int translate_device(gpe_ctx* ctx, const std::vector<uint8_t>* cls, const XlateTabs& T,
                     bool f32, bool typed, uint32_t** d_out, size_t* out_cap,
                     uint32_t** d_start, size_t* start_cap) {
  const int64_t n = ctx->n_prog;
  const auto t_x0 = std::chrono::steady_clock::now();
  const unsigned blocks = (unsigned)((std::max<int64_t>(n, 1) + 255) / 256);
  if (ensure(ctx, &ctx->d_xl_len, &ctx->xl_len_cap, (size_t)n + 1)) return GPE_E_HIP;
  if (ensure(ctx, d_start, start_cap, (size_t)n + 1)) return GPE_E_HIP;
  uint8_t* d_cls = nullptr;
  if (cls) {
    if (ensure(ctx, &ctx->d_xl_cls, &ctx->xl_cls_cap, (size_t)n)) return GPE_E_HIP;
    HIPCHK(hipMemcpyAsync(ctx->d_xl_cls, cls->data(), (size_t)n, hipMemcpyHostToDevice,
                          ctx->stream));
    d_cls = ctx->d_xl_cls;
  }
  uint8_t* d_typed = nullptr;
  if (typed) {
    if (ensure(ctx, &ctx->d_xl_cls, &ctx->xl_cls_cap, (size_t)n)) return GPE_E_HIP;
    d_typed = ctx->d_xl_cls;
  }
  if (ctx->diag) {
    (void)hipStreamSynchronize(ctx->stream);
    fprintf(stderr, "translate_device idle %.3f ms\n",
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_x0)
                .count());
    HIPCHK(hipEventRecord(ctx->ev_redo[0], ctx->stream));
  }
  HIPCHK(hipMemsetAsync(ctx->d_xl_len + n, 0, sizeof(uint32_t), ctx->stream));
  hipLaunchKernelGGL(translate_kernel, dim3(blocks), dim3(256), 0, ctx->stream, ctx->d_code,
                     ctx->d_off, d_cls, n, T, f32 ? 1 : 0, window_use(), 0, ctx->d_xl_len,
                     nullptr, nullptr, d_typed);
  HIPCHK(hipGetLastError());
  if (ctx->diag) {
    HIPCHK(hipEventRecord(ctx->ev_redo[1], ctx->stream));
    (void)hipStreamSynchronize(ctx->stream);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, ctx->ev_redo[0], ctx->ev_redo[1]);
    fprintf(stderr, "translate_device pass 0 on the GPU %.3f ms\n", ms);
  }
  auto xlap = [&](const char* what) {
    if (!ctx->diag) return;
    (void)hipStreamSynchronize(ctx->stream);
    fprintf(stderr, "translate_device %s %.3f ms\n", what,
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_x0)
                .count());
  };
  xlap("pass 0");
  size_t tmp_bytes = 0;
  HIPCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, ctx->d_xl_len, *d_start,
                                          (int)(n + 1), ctx->stream));
  if (ensure(ctx, &ctx->d_sort_tmp, &ctx->sort_tmp_cap, tmp_bytes)) return GPE_E_HIP;
  HIPCHK(hipcub::DeviceScan::ExclusiveSum(ctx->d_sort_tmp, tmp_bytes, ctx->d_xl_len, *d_start,
                                          (int)(n + 1), ctx->stream));
  xlap("scan");
  char* pin = pinned(ctx, 64 + (size_t)n);
  if (!pin) return fail(ctx, GPE_E_HIP, "hipHostMalloc (translation)");
  xlap("pinned");
  HIPCHK(hipMemcpyAsync(pin, *d_start + n, sizeof(uint32_t), hipMemcpyDeviceToHost,
                        ctx->stream));
  if (typed)
    HIPCHK(hipMemcpyAsync(pin + 64, d_typed, (size_t)n, hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  uint32_t total = 0;
  std::memcpy(&total, pin, sizeof(uint32_t));
  if (typed) ctx->typed_ok.assign((const uint8_t*)pin + 64, (const uint8_t*)pin + 64 + n);
  if (ctx->diag)
    fprintf(stderr, "translate_device lengths+scan %.3f ms\n",
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_x0)
                .count());
  const size_t words = (size_t)total + 2 * asmcore::WINDOW;   // s_load_dwordx16 slack
  if (ensure(ctx, d_out, out_cap, words)) return GPE_E_HIP;
  hipLaunchKernelGGL(translate_kernel, dim3(blocks), dim3(256), 0, ctx->stream, ctx->d_code,
                     ctx->d_off, d_cls, n, T, f32 ? 1 : 0, window_use(), 1, ctx->d_xl_len,
                     *d_start, *d_out, d_typed);
  HIPCHK(hipGetLastError());
  const uint32_t end_word = T.tab[typed ? 2 : 0][T.ids[typed ? 2 : 0].H_END];
  std::vector<uint32_t> slack(2 * asmcore::WINDOW, end_word);
  HIPCHK(hipMemcpyAsync(*d_out + total, slack.data(), slack.size() * sizeof(uint32_t),
                        hipMemcpyHostToDevice, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  return 0;
}

// Threaded code of every asm-eligible program for the core of ctx->prec
// (on the first MSE run after a load: other modes never need it),
// translated on the device from the loaded words.
int translate_all(gpe_ctx* ctx) {
  const bool f32 = ctx->prec == GPE_PREC_F32;
  XlateTabs T{};
  T.tab[0] = f32 ? ctx->d_jump_asm32 : ctx->d_jump_asm;
  T.tab[1] = f32 ? ctx->d_jump_asm32_deep : ctx->d_jump_asm_deep;
  T.ids[0] = kIds;
  T.ids[1] = kIdsDeep;
  T.tab[2] = T.tab[0];
  T.ids[2] = kIds;
  int rc = translate_device(ctx, &ctx->asm_ok, T, f32, false, &ctx->d_acode, &ctx->acode_cap,
                            &ctx->d_astart, &ctx->astart_cap);
  if (rc) return rc;
  if (ensure(ctx, &ctx->d_redo, &ctx->redo_cap, (size_t)std::max<int64_t>(ctx->n_prog, 1)))
    return GPE_E_HIP;
  ctx->acode_prec = ctx->prec;
  return 0;
}

// Threaded code of the programs the typed core runs (first HITS_BOOL run
// after a load; the device decides which, typed_runs, and reports them in
// ctx->typed_ok).
int translate_typed(gpe_ctx* ctx) {
  XlateTabs T{};
  for (int t = 0; t < 3; ++t) {
    T.tab[t] = ctx->d_jump_asm_typed;
    T.ids[t] = kIdsTyped;
  }
  int rc = translate_device(ctx, nullptr, T, false, true, &ctx->d_acode_t, &ctx->acode_t_cap,
                            &ctx->d_astart_t, &ctx->astart_t_cap);
  if (rc) return rc;
  ctx->typed_valid = true;
  return 0;
}

}  // namespace
#include "planner.h"
namespace {

// The asm handler table comes from the code object itself (probe launch).
int init_asm(gpe_ctx* ctx) {
  if (ctx->asm_ready) return 0;
  static_assert(kBlock == 64 * 4, "f_eval_asm stages the table per thread");
  std::vector<double> cst(kCstTable + kTrigLdsDoubles, 0.0);
  std::copy(asmcore::kAsmConst, asmcore::kAsmConst + 8, cst.begin());
  // LDS image: the sin table (16-byte entries: random j spread over 16 bank
  // groups), then the polynomial and long-reduction constants
  static_assert(asmcore::SPLIT_TAB == asmcore_deep::SPLIT_TAB,
                "the D = 5 and deep cores read one LDS table image");
  if (asmcore::SPLIT_TAB) {        // hi parts, then lo parts (GEN_ASM_SPLIT_TAB)
    for (int j = 0; j < asmcore::kTrigEntries; ++j) {
      cst[(size_t)kCstTable + j] = asmcore::kTrigTable[2 * j];
      cst[(size_t)kCstTable + asmcore::kTrigEntries + j] = asmcore::kTrigTable[2 * j + 1];
    }
  } else {
    std::copy(asmcore::kTrigTable, asmcore::kTrigTable + 2 * asmcore::kTrigEntries,
              cst.begin() + kCstTable);
  }
  std::copy(asmcore::kTrigLdsTail, asmcore::kTrigLdsTail + 4,
            cst.begin() + kCstTable + 2 * asmcore::kTrigEntries);
  HIPCHK(hipMalloc((void**)&ctx->d_cst, cst.size() * sizeof(double)));
  HIPCHK(hipMemcpy(ctx->d_cst, cst.data(), cst.size() * sizeof(double),
                   hipMemcpyHostToDevice));
  HIPCHK(hipMalloc((void**)&ctx->d_cst32, 16 * sizeof(float)));
  HIPCHK(hipMemcpy(ctx->d_cst32, asmcore32::kConst, 16 * sizeof(float),
                   hipMemcpyHostToDevice));
  {  // the exact core: its two SGPR constant blocks (gen_asm.py GLIBC_SGPR
     // order), then its LDS image: __sincostab, __branred's SPLIT, BBIG1,
     // BMP2 (+ pad), toverp, one pad
    using namespace glibc;
    const double ks[kCstTable] = {HPINV, MP1, MP2, PP3, PP4, BIG, HP0, HP1,
                                  SN3, CS4, CS2, S4, S3, S2, S1, 0.126};
    // __sincostab's image depends on the generator's layout
    // (gen_asm.py GLIBC_TAB_SPLIT): glibc_seq4 reads three 16-byte-stride
    // arrays (sn, ssn) | (cs, ccs) | (-sn, -ssn), GLIBC_SPLIT_S bytes apart
    // (a do_cos lane reads its (A, Aa, B, Bb) at + GLIBC_SPLIT_S); the
    // older bodies read the table as is, then a cos-ordered copy
    // (cs, ccs, -sn, -ssn) after __branred's data
    constexpr int kBr = asmcore_exact::GLIBC_BRANRED_OFF / 8;   // in doubles
    static_assert(asmcore_exact::GLIBC_LDS_BYTES == (kBr + 4 + 75 + 1 +
                                                     (asmcore_exact::GLIBC_TAB_SPLIT ? 0 : 440)) * 8,
                  "LDS image");
    static_assert(asmcore_exact::GLIBC_TAB_SPLIT == asmcore_exact_deep::GLIBC_TAB_SPLIT &&
                      asmcore_exact::GLIBC_BRANRED_OFF == asmcore_exact_deep::GLIBC_BRANRED_OFF,
                  "the exact cores share one LDS image");
    std::vector<double> cx(kCstTable + asmcore_exact::GLIBC_LDS_BYTES / 8, 0.0);
    double* img = cx.data() + kCstTable;
    static_assert(!asmcore_exact::GLIBC_TAB_SPLIT ||
                      (asmcore_exact::GLIBC_SPLIT_S >= 220 * 8 &&
                       3 * asmcore_exact::GLIBC_SPLIT_S <= kBr * 8),
                  "split table arrays");
    if (asmcore_exact::GLIBC_TAB_SPLIT) {
      constexpr int S = asmcore_exact::GLIBC_SPLIT_S / 8;
      for (int e = 0; e < 110; ++e) {
        const double* t = asmcore::kGlibcSincostab + 4 * e;
        img[2 * e] = t[0];                // A: sn, ssn
        img[2 * e + 1] = t[1];
        img[S + 2 * e] = t[2];            // B: cs, ccs
        img[S + 2 * e + 1] = t[3];
        img[2 * S + 2 * e] = -t[0];       // NA: -sn, -ssn
        img[2 * S + 2 * e + 1] = -t[1];
      }
    } else {
      std::copy(asmcore::kGlibcSincostab, asmcore::kGlibcSincostab + 440, img);
      for (int e = 0; e < 110; ++e) {
        const double* t = asmcore::kGlibcSincostab + 4 * e;
        double* c = img + kBr + 80 + 4 * e;
        c[0] = t[2];
        c[1] = t[3];
        c[2] = -t[0];
        c[3] = -t[1];
      }
    }
    std::copy(ks, ks + kCstTable, cx.begin());
    img[kBr] = SPLIT;
    img[kBr + 1] = BBIG1;
    img[kBr + 2] = BMP2;
    std::copy(asmcore::kGlibcToverp, asmcore::kGlibcToverp + 75, img + kBr + 4);
    HIPCHK(hipMalloc((void**)&ctx->d_cst_exact, cx.size() * sizeof(double)));
    HIPCHK(hipMemcpy(ctx->d_cst_exact, cx.data(), cx.size() * sizeof(double),
                     hipMemcpyHostToDevice));
  }
  // the four cores' handler tables (fp64 / fp32, D = 5 / deep; the fp32
  // cores share the fp64 cores' handler lists, with their own offsets)
  static_assert(asmcore32::H_COUNT == asmcore::H_COUNT &&
                    asmcore32::H_BIN0 == asmcore::H_BIN0 &&
                    asmcore32::H_FAM_STRIDE == asmcore::H_FAM_STRIDE &&
                    asmcore32::H_SIN == asmcore::H_SIN &&
                    asmcore32::D == asmcore::D && asmcore32::NV == asmcore::NV,
                "the two asm cores share the handler layout");
  auto probe = [&](auto kern, const auto* cst, int n, std::vector<uint32_t>& out,
                   const char* what) -> int {
    uint32_t* d_tab = nullptr;     // the table, then .Lbase (lo, hi)
    HIPCHK(hipMalloc((void**)&d_tab, (n + 2) * sizeof(uint32_t)));
    hipLaunchKernelGGL(kern, dim3(1), dim3(64), 0, ctx->stream, cst, d_tab);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(ctx->stream));
    out.resize(n);
    HIPCHK(hipMemcpy(out.data(), d_tab, n * sizeof(uint32_t), hipMemcpyDeviceToHost));
    HIPCHK(hipFree(d_tab));
    // handlers are emitted in id order: offsets strictly increase (the
    // first is 0 when the handlers start at the aligned .Lbase)
    for (size_t i = 0; i < out.size(); ++i)
      if (out[i] > (1u << 20) || (out[i] & 3u) || (i && out[i] <= out[i - 1]))
        return fail(ctx, GPE_E_HIP, std::string("implausible ") + what + " handler table");
    return 0;
  };
  int rc;
  if ((rc = probe(f_probe_asm, ctx->d_cst, asmcore::H_COUNT, ctx->asm_table, "asm")))
    return rc;
  if ((rc = probe(f_probe_asm32, ctx->d_cst32, asmcore::H_COUNT, ctx->asm32_table,
                  "fp32 asm")))
    return rc;
  if ((rc = probe(f_probe_asm_deep, ctx->d_cst, asmcore_deep::H_COUNT,
                  ctx->asm_deep_table, "deep asm")))
    return rc;
  static_assert(asmcore_exact::H_COUNT == asmcore::H_COUNT &&
                    asmcore_exact::H_SIN == asmcore::H_SIN &&
                    asmcore_exact::H_BIN0 == asmcore::H_BIN0,
                "the exact core keeps the D = 5 core's handler ids");
  if ((rc = probe(f_probe_asm_exact, ctx->d_cst_exact, asmcore_exact::H_COUNT,
                  ctx->asm_exact_table, "exact asm")))
    return rc;
  HIPCHK(hipMalloc((void**)&ctx->d_redo2_count, sizeof(uint32_t)));
  if ((rc = probe(f_probe_asm32_deep, ctx->d_cst32, asmcore_deep::H_COUNT,
                  ctx->asm32_deep_table, "deep fp32 asm")))
    return rc;
  if ((rc = probe(f_probe_asm_typed, ctx->d_cst, asmcore_typed::H_COUNT,
                  ctx->asm_typed_table, "typed asm")))
    return rc;
  static_assert(asmcore_exact_deep::H_COUNT == asmcore_deep::H_COUNT &&
                    asmcore_exact_deep::H_SIN == asmcore_deep::H_SIN &&
                    asmcore_exact_deep::H_BIN0 == asmcore_deep::H_BIN0,
                "the exact deep core keeps the deep core's handler ids");
  if ((rc = probe(f_probe_asm_exact_deep, ctx->d_cst_exact, asmcore_exact_deep::H_COUNT,
                  ctx->asm_exact_deep_table, "exact deep asm")))
    return rc;
  // each evaluation kernel's own copy of its core: the probe path writes
  // the same offsets and that copy's .Lbase; the jump words are their sum
  // (the high half, shared by all handlers, is set by the core itself)
  auto jumps = [&](auto launch, const std::vector<uint32_t>& rel,
                   std::vector<uint32_t>& out, const char* what) -> int {
    const size_t n = rel.size();
    uint32_t* d_tab = nullptr;
    HIPCHK(hipMalloc((void**)&d_tab, (n + 2) * sizeof(uint32_t)));
    HIPCHK(hipMemsetAsync(d_tab, 0, (n + 2) * sizeof(uint32_t), ctx->stream));
    launch(d_tab);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(ctx->stream));
    std::vector<uint32_t> got(n + 2);
    HIPCHK(hipMemcpy(got.data(), d_tab, (n + 2) * sizeof(uint32_t),
                     hipMemcpyDeviceToHost));
    HIPCHK(hipFree(d_tab));
    const uint64_t base = (uint64_t)got[n] | ((uint64_t)got[n + 1] << 32);
    out.resize(n);
    for (size_t i = 0; i < n; ++i) {
      const uint64_t tgt = base + rel[i];
      if (got[i] != rel[i] || base == 0 || (tgt >> 32) != (base >> 32)) {
        char buf[160];
        snprintf(buf, sizeof(buf), " handler %zu: probed 0x%x, offset 0x%x, base 0x%llx",
                 i, got[i], rel[i], (unsigned long long)base);
        return fail(ctx, GPE_E_HIP, std::string("implausible ") + what +
                                        " handler addresses (table mismatch or a "
                                        "4 GiB boundary inside the core):" + buf);
      }
      out[i] = (uint32_t)tgt;
    }
    return 0;
  };
  // the evaluation kernels reach their core through the normal loop: a
  // one-slot, one-tile task on small scratch buffers (the epilogue after the
  // probe writes there)
  std::vector<char*> scratch;
  auto scratch_buf = [&](size_t bytes) {
    char* p = nullptr;
    if (hipMalloc((void**)&p, bytes) != hipSuccess) return (char*)nullptr;
    (void)hipMemsetAsync(p, 0, bytes, ctx->stream);   // ordered before the probe
    scratch.push_back(p);
    return p;
  };
  auto eval_probe = [&](auto kern, bool exact, bool f32) {
    return [&, kern, exact, f32](uint32_t* d) {
      const int K = f32 ? asmcore32::K : asmcore::K;
      AsmTask t{};
      t.code = (const uint32_t*)scratch_buf(64 * sizeof(uint32_t));
      t.start = (const uint32_t*)scratch_buf(sizeof(uint32_t));
      t.slot_prog = (const int32_t*)scratch_buf(sizeof(int32_t));
      t.n_slots = 1;
      t.P = 1;
      t.X = (const double*)scratch_buf(K * 64 * sizeof(double));
      t.nv = 1;
      t.terms = (const double*)scratch_buf(K * 64 * sizeof(double));
      t.nt = 1;
      t.n_cases = K * 64;
      t.n_tiles = 1;
      t.tiles_per_group = 1;
      t.part = (double*)scratch_buf(2 * sizeof(double));
      t.first_err = (unsigned long long*)scratch_buf(sizeof(unsigned long long));
      t.flags = (uint32_t*)scratch_buf(sizeof(uint32_t));
      t.redo = (uint32_t*)scratch_buf(sizeof(uint32_t));
      t.redo_count = (uint32_t*)scratch_buf(sizeof(uint32_t));
      t.redo_list = (uint64_t*)scratch_buf(sizeof(uint64_t));
      t.redo_list_cap = 1;
      t.cst = exact ? ctx->d_cst_exact : ctx->d_cst;
      t.cst32 = ctx->d_cst32;
      t.redo_hi = ~0u;
      t.base_probe = d;
      const uint32_t tab = f32 ? 0u : exact ? (uint32_t)asmcore_exact::GLIBC_LDS_BYTES
                                            : kTrigLdsBytes;
      const size_t lds = tab + 2 * K * 64 * (f32 ? sizeof(float) : sizeof(double)) +
                         128 * sizeof(double);
      (void)hipFuncSetAttribute((const void*)kern,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      hipLaunchKernelGGL(kern, dim3(1, 1), dim3(64), lds, ctx->stream, t);
    };
  };
  if ((rc = jumps(eval_probe(f_eval_asm<false, false>, false, false), ctx->asm_table,
                  ctx->jump_asm, "asm")) ||
      (rc = jumps(eval_probe(f_eval_asm<false, true>, false, false), ctx->asm_deep_table,
                  ctx->jump_asm_deep, "deep asm")) ||
      (rc = jumps(eval_probe(f_eval_asm<false, false, true>, true, false), ctx->asm_exact_table,
                  ctx->jump_asm_exact, "exact asm")) ||
      (rc = jumps(eval_probe(f_eval_asm<false, true, true>, true, false),
                  ctx->asm_exact_deep_table, ctx->jump_asm_exact_deep, "exact deep asm")) ||
      (rc = jumps(eval_probe(f_eval_asm<true, false>, false, true), ctx->asm32_table,
                  ctx->jump_asm32, "fp32 asm")) ||
      (rc = jumps(eval_probe(f_eval_asm<true, true>, false, true), ctx->asm32_deep_table,
                  ctx->jump_asm32_deep, "deep fp32 asm")) ||
      (rc = jumps([&](uint32_t* d) {
                    constexpr int K = asmcore_typed::K;
                    AsmTask t{};
                    t.code = (const uint32_t*)scratch_buf(64 * sizeof(uint32_t));
                    t.start = (const uint32_t*)scratch_buf(sizeof(uint32_t));
                    t.slot_prog = (const int32_t*)scratch_buf(sizeof(int32_t));
                    t.n_slots = 1;
                    t.P = 1;
                    t.X = (const double*)scratch_buf(K * 64 * sizeof(double));
                    t.nv = 1;
                    t.terms = (const double*)scratch_buf(K * 64 * sizeof(double));
                    t.nt = 1;
                    t.n_cases = K * 64;
                    t.n_tiles = 1;
                    t.tiles_per_group = 1;
                    t.part = (double*)scratch_buf(2 * sizeof(double));
                    t.base_probe = d;
                    hipLaunchKernelGGL(f_eval_asm_typed, dim3(1, 1), dim3(64),
                                       2 * K * 64 * sizeof(double), ctx->stream, t);
                  }, ctx->asm_typed_table, ctx->jump_asm_typed, "typed asm")) ||
      (rc = jumps([&](uint32_t* d) {
                    hipLaunchKernelGGL(asm_values, dim3(1), dim3(64),
                                       kTrigLdsBytes + asmcore::K * 64 * sizeof(double),
                                       ctx->stream,
                                       ctx->d_cst, nullptr, nullptr, nullptr, 0, 0, d);
                  }, ctx->asm_table, ctx->jump_vals, "asm probe")) ||
      (rc = jumps([&](uint32_t* d) {
                    hipLaunchKernelGGL(asm_values_exact, dim3(1), dim3(64),
                                       asmcore_exact::GLIBC_LDS_BYTES +
                                           asmcore_exact::K * 64 * sizeof(double),
                                       ctx->stream,
                                       ctx->d_cst_exact, nullptr, nullptr, nullptr, 0, 0, d);
                  }, ctx->asm_exact_table, ctx->jump_vals_exact, "exact asm probe")) ||
      (rc = jumps([&](uint32_t* d) {
                    hipLaunchKernelGGL(asm_values32, dim3(1), dim3(64),
                                       asmcore32::K * 64 * sizeof(float), ctx->stream,
                                       ctx->d_cst32, nullptr, nullptr, nullptr, 0, 0, d);
                  }, ctx->asm32_table, ctx->jump_vals32, "fp32 asm probe")))
    return rc;
  for (char* p : scratch) HIPCHK(hipFree(p));
  HIPCHK(hipMalloc((void**)&ctx->d_redo_count, sizeof(uint32_t)));
  HIPCHK(hipMalloc((void**)&ctx->d_redo_nsel, sizeof(uint32_t)));
  ctx->redo_list_cap = kRedoListCap;
  // GPE_REDO_CAP: a smaller pair-list capacity (tests force the whole-
  // program redo fallback with it)
  if (const char* cap = getenv("GPE_REDO_CAP"))
    ctx->redo_list_cap = (uint32_t)std::min<long long>(kRedoListCap,
                                                        std::max(0LL, atoll(cap)));
  HIPCHK(hipMalloc((void**)&ctx->d_redo_list, kRedoListCap * sizeof(uint64_t)));
  // the jump words on the device (translate_device)
  auto upload = [&](const std::vector<uint32_t>& v, uint32_t** d) -> int {
    HIPCHK(hipMalloc((void**)d, std::max<size_t>(v.size(), 1) * sizeof(uint32_t)));
    HIPCHK(hipMemcpy(*d, v.data(), v.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
    return 0;
  };
  if (upload(ctx->jump_asm, &ctx->d_jump_asm) ||
      upload(ctx->jump_asm_deep, &ctx->d_jump_asm_deep) ||
      upload(ctx->jump_asm_exact, &ctx->d_jump_asm_exact) ||
      upload(ctx->jump_asm32, &ctx->d_jump_asm32) ||
      upload(ctx->jump_asm32_deep, &ctx->d_jump_asm32_deep) ||
      upload(ctx->jump_asm_typed, &ctx->d_jump_asm_typed) ||
      upload(ctx->jump_asm_exact_deep, &ctx->d_jump_asm_exact_deep))
    return GPE_E_HIP;
  ctx->asm_ready = true;
  return 0;
}

// Build the launch plans for `mode`: MSE on the F machine sends eligible
// programs through the asm core, everything else through the C++ kernels.
int plan_mode(gpe_ctx* ctx, int mode) {
  if (ctx->planned_mode == mode) return 0;
  const bool asm_mode = ctx->machine == GPE_MACHINE_F && mode == GPE_MODE_MSE &&
                        ctx->use_asm && ctx->asm_ready;
  if (asm_mode && ctx->acode_prec != ctx->prec) {
    int rc0 = translate_all(ctx);
    if (rc0) return rc0;
  }
  // HITS_BOOL (fp64): programs the typed core holds run there
  const bool typed_mode = ctx->machine == GPE_MACHINE_F && mode == GPE_MODE_HITS_BOOL &&
                          ctx->use_asm && ctx->use_typed && ctx->asm_ready &&
                          ctx->prec == GPE_PREC_F64 && ctx->nt == 1 && !ctx->case_on;
  if (typed_mode && !ctx->typed_valid) {
    const auto t_x = std::chrono::steady_clock::now();
    int rc0 = translate_typed(ctx);
    if (rc0) return rc0;
    if (ctx->diag)
      fprintf(stderr, "plan_mode translate_typed %.3f ms\n",
              std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_x)
                  .count());
  }
  std::vector<int32_t>&fa = ctx->pl_fa, &da = ctx->pl_da, &ta = ctx->pl_ta, &fc = ctx->pl_fc,
                      &dc = ctx->pl_dc;
  std::vector<int32_t> kc;      // (class 5: constant programs, HITS_BOOL)
  // each program's launch class, in program order within a class (host
  // threads over program ranges at pop 1M: the serial pass was 1-3 ms)
  auto t_p = std::chrono::steady_clock::now();
  {
    const int64_t n = ctx->n_prog;
    auto cls = [&](int64_t i) {
      if (asm_mode && ctx->asm_ok[(size_t)i] == 1) return 0;
      if (asm_mode && ctx->asm_ok[(size_t)i] == 2) return 1;
      if (typed_mode && ctx->typed_ok[(size_t)i]) return ctx->typed_ok[(size_t)i] >= 2 ? 5 : 2;
      return ctx->depth[(size_t)i] <= kFastDepth ? 3 : 4;
    };
    const int nth = n >= 262144 ? host_threads() : 1;
    std::vector<std::array<int64_t, 6>> cnt((size_t)nth);
    hostpool::par_run(nth, [&](int t) {
      std::array<int64_t, 6> c{};
      for (int64_t i = n * t / nth, e = n * (t + 1) / nth; i < e; ++i) ++c[(size_t)cls(i)];
      cnt[(size_t)t] = c;
    });
    std::vector<int32_t>* out[6] = {&fa, &da, &ta, &fc, &dc, &kc};
    for (int k = 0; k < 6; ++k) {
      int64_t run = 0;
      for (int t = 0; t < nth; ++t) {
        const int64_t c = cnt[(size_t)t][(size_t)k];
        cnt[(size_t)t][(size_t)k] = run;
        run += c;
      }
      out[k]->resize((size_t)run);
    }
    hostpool::par_run(nth, [&](int t) {
      std::array<int64_t, 6> at = cnt[(size_t)t];
      for (int64_t i = n * t / nth, e = n * (t + 1) / nth; i < e; ++i) {
        const int k = cls(i);
        (*out[k])[(size_t)at[(size_t)k]++] = (int32_t)i;
      }
    });
  }
  int rc;
  auto lap = [&](const char* what) {
    if (!ctx->diag) return;
    const auto now = std::chrono::steady_clock::now();
    fprintf(stderr, "plan_mode %s %.3f ms\n", what,
            std::chrono::duration<double, std::milli>(now - t_p).count());
    t_p = now;
  };
  lap("classify");
  // the constant programs' list on the device (2 * program + truthy)
  ctx->n_kc = (int64_t)kc.size();
  if (ctx->n_kc) {
    ctx->pl_kc.resize(kc.size());
    for (size_t i = 0; i < kc.size(); ++i)
      ctx->pl_kc[i] = 2u * (uint32_t)kc[i] + (ctx->typed_ok[(size_t)kc[i]] == 3 ? 1u : 0u);
    if (ensure(ctx, &ctx->d_kc, &ctx->kc_cap, kc.size())) return GPE_E_HIP;
    HIPCHK(hipMemcpyAsync(ctx->d_kc, ctx->pl_kc.data(), kc.size() * sizeof(uint32_t),
                          hipMemcpyHostToDevice, ctx->stream));
  }
  if ((rc = plan(ctx, ctx->tasm, ta, false, true, false, true))) return rc;
  lap("typed");
  if ((rc = plan(ctx, ctx->fasm, fa, false, true))) return rc;
  if ((rc = plan(ctx, ctx->dasm, da, false, true, true))) return rc;
  lap("asm");
  if ((rc = plan(ctx, ctx->fast, fc, false, false))) return rc;
  if ((rc = plan(ctx, ctx->deep, dc, true, false))) return rc;
  lap("c++");
  ctx->planned_mode = mode;
  return 0;
}

int launch_cpp(gpe_ctx* ctx, int mode, Launch& fastL, Launch& deepL,
               unsigned long long* err, uint32_t* flags) {
  int rc = 0;
  if (ctx->machine == GPE_MACHINE_F && ctx->prec == GPE_PREC_F32) {
    if (mode == GPE_MODE_MSE) {
      if ((rc = launch_f<kFK32, kFastDepth, GPE_MODE_MSE, float>(ctx, fastL, false, err, flags))) return rc;
      rc = launch_f<1, kDeepDepth, GPE_MODE_MSE, float>(ctx, deepL, true, err, flags);
    } else {
      if ((rc = launch_f<kFK32, kFastDepth, GPE_MODE_HITS_BOOL, float>(ctx, fastL, false, err, flags))) return rc;
      rc = launch_f<1, kDeepDepth, GPE_MODE_HITS_BOOL, float>(ctx, deepL, true, err, flags);
    }
  } else if (ctx->machine == GPE_MACHINE_F) {
    if (mode == GPE_MODE_MSE && ctx->exact_all) {
      // glibc's sin/cos (glibc_trig_k), as the exact asm cores
      if ((rc = launch_f<kFK, kFastDepth, GPE_MODE_MSE, double, true>(ctx, fastL, false, err,
                                                                        flags)))
        return rc;
      rc = launch_f<1, kDeepDepth, GPE_MODE_MSE, double, true>(ctx, deepL, true, err, flags);
    } else if (mode == GPE_MODE_MSE) {
      if ((rc = launch_f<kFK, kFastDepth, GPE_MODE_MSE, double>(ctx, fastL, false, err, flags))) return rc;
      rc = launch_f<1, kDeepDepth, GPE_MODE_MSE, double>(ctx, deepL, true, err, flags);
    } else {
      if ((rc = launch_f<kFK, kFastDepth, GPE_MODE_HITS_BOOL, double>(ctx, fastL, false, err, flags))) return rc;
      rc = launch_f<1, kDeepDepth, GPE_MODE_HITS_BOOL, double>(ctx, deepL, true, err, flags);
    }
  } else {
    if ((rc = launch_b<kFastDepth>(ctx, fastL, false))) return rc;
    rc = launch_b<kDeepDepth>(ctx, deepL, true);
  }
  return rc;
}

}  // namespace
#include "exact_run.h"
namespace {

int run_common(gpe_ctx* ctx, int mode, double* hi, double* lo,
               unsigned long long* err, uint32_t* flags) {
  if (ctx->machine < 0) return fail(ctx, GPE_E_STATE, "gpe_set_cases not called");
  if (ctx->n_prog <= 0) return 0;
  const bool F = ctx->machine == GPE_MACHINE_F;
  if (F && mode == GPE_MODE_HITS_BITS)
    return fail(ctx, GPE_E_INVALID, "HITS_BITS needs the B machine");
  if (!F && mode != GPE_MODE_HITS_BITS)
    return fail(ctx, GPE_E_INVALID, "the B machine only supports HITS_BITS");
  if (F && mode == GPE_MODE_MSE && ctx->nt < 1)
    return fail(ctx, GPE_E_INVALID, "MSE needs at least one target term");
  int rc;
  ctx->last_mode = -1;         // the entry points re-validate on success
  const auto t_r0 = std::chrono::steady_clock::now();
  if ((rc = plan_mode(ctx, mode))) return rc;
  if (ctx->diag)
    fprintf(stderr, "run_common plan %.3f ms\n",
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_r0)
                .count());
  HIPCHK(hipMemsetAsync(err, 0xff, ctx->n_prog * sizeof(unsigned long long), ctx->stream));
  HIPCHK(hipMemsetAsync(flags, 0, ctx->n_prog * sizeof(uint32_t), ctx->stream));
  const bool any_asm = ctx->fasm.n_slots || ctx->dasm.n_slots;
  if (any_asm) {
    HIPCHK(hipMemsetAsync(ctx->d_redo, 0, ctx->n_prog * sizeof(uint32_t), ctx->stream));
    HIPCHK(hipMemsetAsync(ctx->d_redo_count, 0, sizeof(uint32_t), ctx->stream));
  }
  HIPCHK(hipEventRecord(ctx->ev[0], ctx->stream));
  if (ctx->trig_leaves) {
    const int64_t n = ctx->n_cases * ctx->nv_user;
    hipLaunchKernelGGL(leaf_trig, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       ctx->stream, (double*)ctx->d_X, ctx->nv_user, ctx->n_cases,
                       ctx->prec == GPE_PREC_F32 ? 1 : 0);
    HIPCHK(hipGetLastError());
  }
  // every D <= 12 asm program on the exact cores (glibc's sin/cos in the
  // handlers: the reference's math.sin/cos bit for bit) instead of the
  // table cores (GPE_EXACT_ALL=0: the table cores and their redo pass)
  const bool exact_all = ctx->exact_all && F && mode == GPE_MODE_MSE &&
                         ctx->prec == GPE_PREC_F64 &&
                         (ctx->fasm.n_slots || ctx->dasm.n_slots);
  ctx->last_exact_all = exact_all;
  if (exact_all) {
    std::vector<int32_t> rx, rxd, rest;
    for (int64_t i = 0; i < ctx->fasm.n_slots; ++i)
      if (ctx->fasm.slot_prog[(size_t)i] >= 0) rx.push_back(ctx->fasm.slot_prog[(size_t)i]);
    for (int64_t i = 0; i < ctx->dasm.n_slots; ++i)
      if (ctx->dasm.slot_prog[(size_t)i] >= 0) rxd.push_back(ctx->dasm.slot_prog[(size_t)i]);
    std::sort(rx.begin(), rx.end());
    std::sort(rxd.begin(), rxd.end());
    if ((rc = run_exact_asm(ctx, rx, hi, lo, err, flags, rest, rxd))) return rc;
    if (!rest.empty()) {
      if ((rc = plan(ctx, ctx->redo_fast, rest, false, false))) return rc;
      if ((rc = launch_f<kFK, kFastDepth, GPE_MODE_MSE, double, true>(
               ctx, ctx->redo_fast, false, err, flags)))
        return rc;
      if ((rc = launch_reduce(ctx, ctx->redo_fast, hi, lo))) return rc;
    }
  } else if ((rc = launch_asm(ctx, ctx->fasm, err, flags))) {
    return rc;
  }
  if (!exact_all && (rc = launch_asm(ctx, ctx->dasm, err, flags, true))) return rc;
  if ((rc = launch_asm_typed(ctx, ctx->tasm))) return rc;
  if (ctx->n_kc && mode == GPE_MODE_HITS_BOOL) {
    const int64_t nk = ctx->n_kc;
    hipLaunchKernelGGL(const_hits, dim3((unsigned)((nk + 255) / 256)), dim3(256), 0, ctx->stream,
                       ctx->d_kc, nk, (double)ctx->label_true,
                       (double)(ctx->n_cases - ctx->label_true), hi, lo);
    HIPCHK(hipGetLastError());
  }
  if ((rc = launch_cpp(ctx, mode, ctx->fast, ctx->deep, err, flags))) return rc;
  HIPCHK(hipEventRecord(ctx->ev[1], ctx->stream));
  if ((rc = launch_reduce(ctx, ctx->tasm, hi, lo))) return rc;
  if (!exact_all && (rc = launch_reduce(ctx, ctx->fasm, hi, lo))) return rc;
  if (!exact_all && (rc = launch_reduce(ctx, ctx->dasm, hi, lo))) return rc;
  if ((rc = launch_reduce(ctx, ctx->fast, hi, lo))) return rc;
  if ((rc = launch_reduce(ctx, ctx->deep, hi, lo))) return rc;
  HIPCHK(hipEventRecord(ctx->ev[2], ctx->stream));
  ctx->redo_programs = 0;
  ctx->redo_tiles = 0;
  ctx->redo_exact_cpp = 0;
  // the redo bookkeeping rides the same stream as the main pass: (sharded)
  // the flags' all-reduce, the flagged programs compacted on the device in
  // program order, and ONE pinned D2H of [flagged tiles, flagged programs,
  // the list's first kRedoHead entries] — one host sync for all of it
  constexpr int64_t kRedoHead = 4096;
  const uint32_t* rpin = nullptr;
  if (any_asm) {
    if (!ctx->debug_redo_or.empty() && ctx->prec == GPE_PREC_F64) {
      // the union the all-reduce below forms, with the other ranks' flags
      // given by the test: OR them in and count them as flagged tiles
      HIPCHK(hipStreamSynchronize(ctx->stream));
      const int64_t m = std::min<int64_t>(ctx->n_prog, (int64_t)ctx->debug_redo_or.size());
      std::vector<uint32_t> mine((size_t)ctx->n_prog);
      HIPCHK(hipMemcpy(mine.data(), ctx->d_redo, ctx->n_prog * sizeof(uint32_t),
                       hipMemcpyDeviceToHost));
      uint32_t extra = 0;
      for (int64_t i = 0; i < m; ++i)
        if (ctx->debug_redo_or[(size_t)i] && !mine[(size_t)i]) {
          mine[(size_t)i] = 1;
          ++extra;
        }
      HIPCHK(hipMemcpy(ctx->d_redo, mine.data(), ctx->n_prog * sizeof(uint32_t),
                       hipMemcpyHostToDevice));
      uint32_t cnt0 = 0;
      HIPCHK(hipMemcpy(&cnt0, ctx->d_redo_count, sizeof(uint32_t), hipMemcpyDeviceToHost));
      cnt0 += extra;
      HIPCHK(hipMemcpy(ctx->d_redo_count, &cnt0, sizeof(uint32_t), hipMemcpyHostToDevice));
    }
    // (the exact cores raise no redo flag: nothing to combine)
    ctx->redo_timed = false;
    if (ctx->redo_global && ctx->comm && ctx->prec == GPE_PREC_F64 && !exact_all) {
      // case-sharded (gpe_run_sharded*): a program flagged on any rank is
      // re-run whole on every rank, so its fitness does not depend on how
      // the cases were split
      RcclApi& r = rccl();
      HIPCHK(hipEventRecord(ctx->ev_comm[2], ctx->stream));
      ncclResult_t e1 = r.all_reduce(ctx->d_redo, ctx->d_redo, (size_t)ctx->n_prog,
                                     ncclUint32, ncclMax, ctx->comm, ctx->stream);
      ncclResult_t e2 = r.all_reduce(ctx->d_redo_count, ctx->d_redo_count, 1,
                                     ncclUint32, ncclSum, ctx->comm, ctx->stream);
      HIPCHK(hipEventRecord(ctx->ev_comm[3], ctx->stream));
      ctx->redo_timed = true;
      if (e1 != ncclSuccess || e2 != ncclSuccess)
        return fail(ctx, GPE_E_HIP, std::string("redo flags all-reduce: ") +
                                        r.error_string(e1 != ncclSuccess ? e1 : e2));
    }
    const int n = (int)ctx->n_prog;
    if (ensure(ctx, &ctx->d_redo_progs, &ctx->redo_progs_cap, (size_t)n)) return GPE_E_HIP;
    hipcub::CountingInputIterator<int32_t> ids(0);
    size_t tmp_bytes = 0;
    HIPCHK(hipcub::DeviceSelect::Flagged(nullptr, tmp_bytes, ids, ctx->d_redo,
                                         ctx->d_redo_progs, ctx->d_redo_nsel, n,
                                         ctx->stream));
    if (ensure(ctx, &ctx->d_sort_tmp, &ctx->sort_tmp_cap, tmp_bytes)) return GPE_E_HIP;
    HIPCHK(hipcub::DeviceSelect::Flagged(ctx->d_sort_tmp, tmp_bytes, ids, ctx->d_redo,
                                         ctx->d_redo_progs, ctx->d_redo_nsel, n,
                                         ctx->stream));
    uint32_t* pin = (uint32_t*)pinned_buf(&ctx->h_pin_redo, &ctx->h_pin_redo_cap,
                                          (2 + kRedoHead) * sizeof(uint32_t));
    if (!pin) return fail(ctx, GPE_E_HIP, "pinned redo readback buffer");
    HIPCHK(hipMemcpyAsync(pin, ctx->d_redo_count, sizeof(uint32_t), hipMemcpyDeviceToHost,
                          ctx->stream));
    HIPCHK(hipMemcpyAsync(pin + 1, ctx->d_redo_nsel, sizeof(uint32_t),
                          hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipMemcpyAsync(pin + 2, ctx->d_redo_progs,
                          (size_t)std::min<int64_t>(n, kRedoHead) * sizeof(int32_t),
                          hipMemcpyDeviceToHost, ctx->stream));
    rpin = pin;
  }
  if (ctx->redo_timed) {
    if ((rc = comm_sync(ctx, "redo-flag all-reduce"))) return rc;
  } else {
    HIPCHK(hipStreamSynchronize(ctx->stream));
  }
  HIPCHK(hipEventElapsedTime(&ctx->ms[0], ctx->ev[0], ctx->ev[1]));
  HIPCHK(hipEventElapsedTime(&ctx->ms[1], ctx->ev[1], ctx->ev[2]));
  ctx->ms[2] = ctx->ms[0] + ctx->ms[1];
  if (any_asm) {
    const uint32_t cnt = rpin[0];
    const int64_t nsel = (int64_t)rpin[1];
    ctx->redo_tiles = cnt;
    if (cnt) HIPCHK(hipEventRecord(ctx->ev_redo[0], ctx->stream));
    // fp64: every flagged program is re-run whole with the reference's own
    // sin/cos (glibc_trig): a sin/cos argument past 2^40 marks a program
    // whose value is chaotic in the last bits of its intermediates, so all
    // of its cases must round as the reference's libm does (re-running only
    // the flagged tiles left 4 of the 48 bench-sample trees 1e-10 off).
    // fp32 (approximate mode): only the flagged (program, tile) pairs.
    if (cnt && ctx->prec == GPE_PREC_F32 && cnt <= ctx->redo_list_cap) {
      if ((rc = redo_pairs(ctx, cnt, hi, lo, err, flags))) return rc;
    } else if (cnt) {
      // re-run the flagged programs whole with the C++ kernels (fp64: with
      // glibc_trig for every sin/cos)
      std::vector<int32_t> list((size_t)nsel);
      if (nsel <= kRedoHead)
        std::memcpy(list.data(), rpin + 2, (size_t)nsel * sizeof(int32_t));
      else   // the stream is idle: a plain copy of the whole list
        HIPCHK(hipMemcpy(list.data(), ctx->d_redo_progs, (size_t)nsel * sizeof(int32_t),
                         hipMemcpyDeviceToHost));
      std::vector<int32_t> rf, rd;
      for (int32_t i : list) (ctx->depth[(size_t)i] <= kFastDepth ? rf : rd).push_back(i);
      ctx->redo_programs = nsel;
      hipLaunchKernelGGL(clear_entries, dim3((unsigned)((nsel + 255) / 256)),
                         dim3(256), 0, ctx->stream, ctx->d_redo_progs, nsel, err, flags);
      HIPCHK(hipGetLastError());
      if (mode == GPE_MODE_MSE && ctx->prec == GPE_PREC_F64 && ctx->use_asm) {
        // stage 1: programs the D = 5 core holds run on the exact core
        // (glibc's sin/cos in the handlers); those with a lane it leaves
        // (|x| >= 105414350, inf, nan) join the C++ pass below
        // (the deep core's programs on the exact deep core)
        std::vector<int32_t> rx, rxd, rc2, rd2;
        for (int32_t i : rf)
          (ctx->asm_ok[(size_t)i] == 1 ? rx : ctx->asm_ok[(size_t)i] == 2 ? rxd : rc2)
              .push_back(i);
        for (int32_t i : rd) (ctx->asm_ok[(size_t)i] == 2 ? rxd : rd2).push_back(i);
        if (!rx.empty() || !rxd.empty()) {
          // programs the exact cores leave (a lane past glibc's range) come
          // back in rc2 for the C++ exact kernels, by depth
          std::vector<int32_t> back;
          if ((rc = run_exact_asm(ctx, rx, hi, lo, err, flags, back, rxd))) return rc;
          for (int32_t i : back) (ctx->depth[(size_t)i] <= kFastDepth ? rc2 : rd2).push_back(i);
          rf.swap(rc2);
          rd.swap(rd2);
        }
      }
      if ((rc = plan(ctx, ctx->redo_fast, rf, false, false))) return rc;
      if ((rc = plan(ctx, ctx->redo_deep, rd, true, false))) return rc;
      if (mode == GPE_MODE_MSE && ctx->prec == GPE_PREC_F64) {
        // the pair pass's arithmetic: glibc_trig for every sin/cos
        if ((rc = launch_f<kFK, kFastDepth, GPE_MODE_MSE, double, true>(
                 ctx, ctx->redo_fast, false, err, flags)))
          return rc;
        if ((rc = launch_f<1, kDeepDepth, GPE_MODE_MSE, double, true>(
                 ctx, ctx->redo_deep, true, err, flags)))
          return rc;
      } else if ((rc = launch_cpp(ctx, mode, ctx->redo_fast, ctx->redo_deep, err,
                                  flags))) {
        return rc;
      }
      if ((rc = launch_reduce(ctx, ctx->redo_fast, hi, lo))) return rc;
      if ((rc = launch_reduce(ctx, ctx->redo_deep, hi, lo))) return rc;
      HIPCHK(hipStreamSynchronize(ctx->stream));
    }
    if (cnt) {                 // the redo passes count as interpreter time
      HIPCHK(hipEventRecord(ctx->ev_redo[1], ctx->stream));
      HIPCHK(hipEventSynchronize(ctx->ev_redo[1]));
      float ms = 0.0f;
      HIPCHK(hipEventElapsedTime(&ms, ctx->ev_redo[0], ctx->ev_redo[1]));
      ctx->ms[0] += ms;
      ctx->ms[2] += ms;
    }
  }
  if (ctx->ex_all > 0 && F && ctx->prec == GPE_PREC_F64 &&
      (mode == GPE_MODE_MSE || mode == GPE_MODE_HITS_BOOL)) {
    if ((rc = run_exact(ctx, mode, hi, lo, err, flags))) return rc;
  }
  return 0;
}

}  // namespace

extern "C" {

int gpe_create(int device, gpe_ctx** out) {
  if (!out) return GPE_E_INVALID;
  *out = nullptr;
  gpe_ctx* ctx = new gpe_ctx();
  ctx->device = device;
  const char* env = getenv("GPE_ASM");
  if (env && env[0] == '0') ctx->use_asm = 0;
  // tuning knobs (experiments; defaults are the tuned values)
  if ((env = getenv("GPE_ASM_P")) && atoi(env) >= 1 && atoi(env) <= 16)
    ctx->asm_pmax = atoi(env);
  if ((env = getenv("GPE_TARGET_BLOCKS")) && atol(env) >= 256)
    ctx->target_blocks = atol(env);
  if ((env = getenv("GPE_ASM_TARGET_BLOCKS")) && atol(env) >= 256)
    ctx->asm_target_blocks = atol(env);
  if ((env = getenv("GPE_TYPED_TARGET_BLOCKS")) && atol(env) >= 256)
    ctx->typed_target_blocks = atol(env);
  if ((env = getenv("GPE_MIN_GROUP_TILES")) && atol(env) >= 0)
    ctx->min_group_tiles = atol(env);
  if ((env = getenv("GPE_XASM_TARGET_BLOCKS")) && atol(env) >= 64)
    ctx->xasm_target_blocks = atol(env);
  if ((env = getenv("GPE_TRIG_W")) && atoi(env) >= 0 && atoi(env) <= 1000)
    ctx->trig_w = atoi(env);
  if ((env = getenv("GPE_DEAL_MIX"))) ctx->deal_mix = atoi(env);
  if ((env = getenv("GPE_DIV_W")) && atoi(env) >= 0 && atoi(env) <= 1000)
    ctx->div_w = atoi(env);
  if ((env = getenv("GPE_DIAG"))) ctx->diag = atoi(env);
  if ((env = getenv("GPE_EXACT_ALL"))) ctx->exact_all = atoi(env) != 0;
  if ((env = getenv("GPE_REDO_EXP")) && atoi(env) >= 14 && atoi(env) <= 40)
    ctx->redo_hi = (uint32_t)(0x3ff + atoi(env)) << 20;
  if ((env = getenv("GPE_REDO_EXP_DEEP")) && atoi(env) >= 14 && atoi(env) <= 40)
    ctx->redo_hi_deep = (uint32_t)(0x3ff + atoi(env)) << 20;
  if ((env = getenv("GPE_ASM_WAVES")) && atoi(env) >= 2 &&
      atoi(env) * 64 <= kAsmMaxBlock)
    ctx->asm_waves = atoi(env);
  if ((env = getenv("GPE_ASM_LDS_KB")) && atoi(env) >= 16 && atoi(env) <= 160)
    ctx->asm_lds_kb = atoi(env);
  if ((env = getenv("GPE_ASM_DBUF"))) ctx->asm_dbuf = atoi(env) != 0;
  if ((env = getenv("GPE_LOWER_IL"))) ctx->lw_interleave = atoi(env) != 0;
  if ((env = getenv("GPE_NEG_PEEPHOLE"))) ctx->neg_fold = atoi(env) != 0;
  if ((env = getenv("GPE_ASM_DEEP_WAVES")) && (atoi(env) == 4 || atoi(env) == 8))
    ctx->asm_deep_waves = atoi(env);
  if ((env = getenv("GPE_F_WAVES")) && (atoi(env) == 4 || atoi(env) == 8))
    ctx->f_waves = atoi(env);
  if ((env = getenv("GPE_B_LANES"))) ctx->b_lanes = atoi(env) != 0;
  if ((env = getenv("GPE_TYPED_ASM"))) ctx->use_typed = atoi(env) != 0;
  if ((env = getenv("GPE_TYPED_PMAX")) && atoi(env) >= 1 && atoi(env) <= 64)
    ctx->typed_pmax = atoi(env);
  if ((env = getenv("GPE_TYPED_WAVES")) && atoi(env) >= 1 && atoi(env) <= 16)
    ctx->typed_waves = atoi(env);
  auto init = [&]() -> int {
    HIPCHK(hipSetDevice(device));
    HIPCHK(hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking));
    for (auto& e : ctx->ev) HIPCHK(hipEventCreate(&e));
    for (auto& e : ctx->ev_redo) HIPCHK(hipEventCreate(&e));
    HIPCHK(hipEventCreateWithFlags(&ctx->ev_lw, hipEventDisableTiming));
    hipDeviceProp_t prop;
    HIPCHK(hipGetDeviceProperties(&prop, device));
    ctx->cu = prop.multiProcessorCount;
    ctx->clock_khz = prop.clockRate;
    snprintf(ctx->name, sizeof(ctx->name), "%s", prop.gcnArchName);
    if (ctx->use_asm) return init_asm(ctx);
    return 0;
  };
  int rc = init();
  if (rc) {
    fprintf(stderr, "gpe_create: %s\n", ctx->err.c_str());
    gpe_destroy(ctx);
    return rc;
  }
  *out = ctx;
  return 0;
}

void gpe_destroy(gpe_ctx* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  void* bufs[] = {ctx->d_X, ctx->d_terms, ctx->d_code, ctx->d_off,
                  ctx->fast.d_slot_prog, ctx->fast.d_part,
                  ctx->deep.d_slot_prog, ctx->deep.d_part,
                  ctx->fasm.d_slot_prog, ctx->fasm.d_part,
                  ctx->dasm.d_slot_prog, ctx->dasm.d_part,
                  ctx->redo_fast.d_slot_prog, ctx->redo_fast.d_part,
                  ctx->redo_deep.d_slot_prog, ctx->redo_deep.d_part,
                  ctx->redo_xasm.d_slot_prog, ctx->redo_xasm.d_part,
                  ctx->d_cst_exact, ctx->d_acode_x, ctx->d_astart_x, ctx->d_redo2,
                  ctx->d_redo2_count, ctx->d_lw_entries, ctx->d_lw_leaf, ctx->d_lw_nw,
                  ctx->d_lw_meta,
                  ctx->d_hi, ctx->d_lo, ctx->d_err, ctx->d_flags, ctx->d_cst,
                  ctx->d_acode, ctx->d_astart, ctx->d_redo, ctx->d_redo_count,
                  ctx->d_redo_list, ctx->d_pair_part, ctx->d_pair_sorted,
                  ctx->d_cst32,
                  ctx->d_pair_off, ctx->d_pair_nruns, ctx->d_sort_tmp,
                  ctx->d_case_out, ctx->d_np_off, ctx->d_np_len,
                  ctx->d_np_post, ctx->d_np_leaf, ctx->d_pair,
                  ctx->d_gather, ctx->d_pack, ctx->d_tags, ctx->d_ncount,
                  ctx->d_sel_wv, ctx->d_sel_draws, ctx->d_sel_out, ctx->d_sel_state,
                  ctx->d_lex_val, ctx->d_lex_max, ctx->d_lex_status, ctx->d_lex_scratch,
                  ctx->d_redo_progs, ctx->d_ex_progs, ctx->d_ex_code, ctx->d_ex_off,
                  ctx->d_ex_ints, ctx->d_ex_rows,
                  ctx->tasm.d_slot_prog, ctx->tasm.d_part,
                  ctx->redo_xasm_deep.d_slot_prog, ctx->redo_xasm_deep.d_part,
                  ctx->d_acode_t, ctx->d_astart_t, ctx->d_xl_len, ctx->d_xl_cls,
                  ctx->d_jump_asm, ctx->d_jump_asm_deep, ctx->d_jump_asm_exact,
                  ctx->d_jump_asm32, ctx->d_jump_asm32_deep, ctx->d_jump_asm_typed,
                  ctx->d_jump_asm_exact_deep, ctx->d_redo_nsel, ctx->d_kc, ctx->d_exh_rec};
  if (ctx->comm && rccl().ok) (void)rccl().comm_destroy(ctx->comm);
  for (void* b : bufs)
    if (b) (void)hipFree(b);
  if (ctx->h_pin) (void)hipHostFree(ctx->h_pin);
  if (ctx->h_pin_in) (void)hipHostFree(ctx->h_pin_in);
  if (ctx->h_pin_redo) (void)hipHostFree(ctx->h_pin_redo);
  for (LowerChunk& C : ctx->lw_ch) {
    for (void* b : std::initializer_list<void*>{C.codes, C.node_off, C.eph_off, C.evals, C.l16,
                                                 C.rec, C.stk, C.cv, C.ib, C.words, C.wrow,
                                                 C.wword})
      if (b) (void)hipFree(b);
    if (C.h_pin) (void)hipHostFree(C.h_pin);
    if (C.ev) (void)hipEventDestroy(C.ev);
    if (C.scan_tmp) (void)hipFree(C.scan_tmp);
  }
  for (hipStream_t st : ctx->lw_stream)
    if (st) (void)hipStreamDestroy(st);
  if (ctx->lw_hm) (void)hipHostFree(ctx->lw_hm);
  for (Launch* L : {&ctx->fast, &ctx->deep, &ctx->fasm, &ctx->dasm, &ctx->tasm, &ctx->redo_fast,
                    &ctx->redo_deep, &ctx->redo_xasm, &ctx->redo_xasm_deep})
    if (L->h_pin) (void)hipHostFree(L->h_pin);
  for (auto& e : ctx->ev)
    if (e) (void)hipEventDestroy(e);
  for (auto& e : ctx->ev_redo)
    if (e) (void)hipEventDestroy(e);
  if (ctx->ev_lw) (void)hipEventDestroy(ctx->ev_lw);
  for (auto& e : ctx->ev_comm)
    if (e) (void)hipEventDestroy(e);
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  delete ctx;
}

const char* gpe_last_error(const gpe_ctx* ctx) {
  return ctx ? ctx->err.c_str() : "null context";
}

int gpe_device_info(const gpe_ctx* ctx, int* n_cu, int* clock_khz, char* name,
                    size_t name_len) {
  if (!ctx) return GPE_E_INVALID;
  if (n_cu) *n_cu = ctx->cu;
  if (clock_khz) *clock_khz = ctx->clock_khz;
  if (name && name_len) snprintf(name, name_len, "%s", ctx->name);
  return 0;
}

int gpe_set_cases(gpe_ctx* ctx, int machine, const void* X, int n_vars,
                  int64_t n_cases, const void* terms, int n_terms) {
  if (!ctx) return GPE_E_INVALID;
  ctx->last_mode = -1;         // resident fitness no longer matches
  ctx->n_exact = 0;            // the exact pass belongs to a population
  ctx->ex_all = 0;
  if (machine != GPE_MACHINE_F && machine != GPE_MACHINE_B)
    return fail(ctx, GPE_E_INVALID, "unknown machine");
  if (n_vars < 0 || n_cases <= 0 || n_terms < 0 || (n_vars > 0 && !X))
    return fail(ctx, GPE_E_INVALID, "bad case arrays");
  if (machine == GPE_MACHINE_B && !terms)
    return fail(ctx, GPE_E_INVALID, "B machine needs the output plane");
  HIPCHK(hipSetDevice(ctx->device));
  if (ctx->d_X) HIPCHK(hipFree(ctx->d_X));
  if (ctx->d_terms) HIPCHK(hipFree(ctx->d_terms));
  ctx->d_X = ctx->d_terms = nullptr;
  ctx->machine = machine;
  ctx->nv = ctx->nv_user = n_vars;
  ctx->trig_leaves = 0;
  ctx->n_cases = n_cases;
  ctx->ex_hcases = false;      // (the host exact pass copies them on need)
  ctx->n_prog = 0;
  ctx->planned_mode = -1;
  size_t xb, tb;
  if (machine == GPE_MACHINE_F) {
    ctx->nt = n_terms;
    ctx->n_units = n_cases;
    xb = (size_t)n_vars * n_cases * sizeof(double);
    tb = (size_t)n_terms * n_cases * sizeof(double);
  } else {
    ctx->nt = 1;
    ctx->n_units = (n_cases + 31) / 32;
    xb = (size_t)n_vars * ctx->n_units * sizeof(uint32_t);
    tb = (size_t)ctx->n_units * sizeof(uint32_t);
  }
  if (lds_bytes(ctx, true) > 160 * 1024 || lds_bytes(ctx, false) > 160 * 1024)
    return fail(ctx, GPE_E_INVALID, "too many variables for one LDS tile");
  HIPCHK(hipMalloc(&ctx->d_X, std::max<size_t>(xb, 8)));
  HIPCHK(hipMalloc(&ctx->d_terms, std::max<size_t>(tb, 8)));
  if (xb) HIPCHK(hipMemcpy(ctx->d_X, X, xb, hipMemcpyHostToDevice));
  if (tb) HIPCHK(hipMemcpy(ctx->d_terms, terms, tb, hipMemcpyHostToDevice));
  if (machine == GPE_MACHINE_F && xb) {
    // every NaN of the cases as the default NaN (low word 0): the asm
    // cores' protectedDiv selects only the high word of 1.0 for den == 0,
    // which needs the fixup's NaN (a NaN numerator's own) to have low word 0
    const int64_t n = (int64_t)n_vars * n_cases;
    hipLaunchKernelGGL(canon_nan, dim3((unsigned)std::min<int64_t>((n + 255) / 256, 65536)),
                       dim3(256), 0, ctx->stream, (double*)ctx->d_X, n);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(ctx->stream));
  }
  // the first target column's truths (HITS_BOOL: a constant program's hits)
  ctx->label_true = 0;
  if (machine == GPE_MACHINE_F && n_terms >= 1) {
    const double* lab = (const double*)terms;
    int64_t t = 0;
    for (int64_t c = 0; c < n_cases; ++c) t += lab[c] != 0.0;
    ctx->label_true = t;
  }
  return 0;
}

int gpe_set_trig_leaves(gpe_ctx* ctx, int enable) {
  if (!ctx) return GPE_E_INVALID;
  ctx->last_mode = -1;         // resident fitness no longer matches
  if (ctx->machine != GPE_MACHINE_F)
    return fail(ctx, GPE_E_STATE, "trig leaves need F-machine cases");
  HIPCHK(hipSetDevice(ctx->device));
  const int want = enable ? 3 * ctx->nv_user : ctx->nv_user;
  if (want != ctx->nv) {
    const size_t col = (size_t)ctx->n_cases * sizeof(double);
    if (enable) {
      const int nv0 = ctx->nv;
      ctx->nv = want;
      if (lds_bytes(ctx, true) > 160 * 1024 || lds_bytes(ctx, false) > 160 * 1024 ||
          lds_bytes_asm(ctx, 1, kWaves, asmcore::K, false) > 160 * 1024) {
        ctx->nv = nv0;
        return fail(ctx, GPE_E_INVALID, "too many variables for trig leaves");
      }
      void* d = nullptr;
      HIPCHK(hipMalloc(&d, std::max<size_t>(col * want, 8)));
      HIPCHK(hipMemcpy(d, ctx->d_X, col * ctx->nv_user, hipMemcpyDeviceToDevice));
      HIPCHK(hipFree(ctx->d_X));
      ctx->d_X = d;
    }
    ctx->nv = want;          // shrinking keeps the allocation
  }
  ctx->trig_leaves = enable ? 1 : 0;
  ctx->n_prog = 0;           // programs were validated against the old nv
  ctx->planned_mode = -1;
  return 0;
}

int gpe_set_lowering(gpe_ctx* ctx, int machine, int nv, const uint8_t* leaf,
                     int n_leaf, const gpe_entry* entries, int n_entries) {
  if (!ctx || (machine != GPE_MACHINE_F && machine != GPE_MACHINE_B) || nv < 0 ||
      n_leaf < 0 || (n_leaf && !leaf) || n_entries <= 0 || n_entries >= 255 || !entries)
    return GPE_E_INVALID;
  HIPCHK(hipSetDevice(ctx->device));
  if (ctx->d_lw_entries) HIPCHK(hipFree(ctx->d_lw_entries));
  if (ctx->d_lw_leaf) HIPCHK(hipFree(ctx->d_lw_leaf));
  ctx->d_lw_entries = nullptr;
  ctx->d_lw_leaf = nullptr;
  HIPCHK(hipMalloc((void**)&ctx->d_lw_entries, n_entries * sizeof(lowering::Entry)));
  HIPCHK(hipMemcpy(ctx->d_lw_entries, entries, n_entries * sizeof(lowering::Entry),
                   hipMemcpyHostToDevice));
  HIPCHK(hipMalloc((void**)&ctx->d_lw_leaf, (size_t)std::max(n_leaf, 1)));
  if (n_leaf)
    HIPCHK(hipMemcpy(ctx->d_lw_leaf, leaf, (size_t)n_leaf, hipMemcpyHostToDevice));
  ctx->lw_machine = machine;
  ctx->lw_nv = nv;
  ctx->lw_n_leaf = n_leaf;
  return 0;
}

}  // extern "C"

namespace {

// ensure() with headroom: the chunk buffers change size with the trees
template <typename T>
int ensure_slack(gpe_ctx* ctx, T** ptr, size_t* cap, size_t n) {
  if (n <= *cap && *ptr) return 0;
  return ensure(ctx, ptr, cap, n + n / 4);
}


// The per-program pass over trees [a, a + n) of the open lowering, from the
// word counts and metadata lower_trees wrote (copied back into ctx->lw_hm):
// what gpe_load_programs derives from validated words, and the caller's
// depth / error / status (every entry is written: the vectors are resized at
// gpe_lower_begin, not refilled).
void decode_lowered(gpe_ctx* ctx, int64_t a, int64_t n, int32_t* out_depth, uint8_t* out_err,
                    uint8_t* out_status) {
  const uint32_t* nw = ctx->lw_hm;
  const uint32_t* meta = ctx->lw_hm + ctx->lw_total_n;
  // (all host threads also inside gpe_lower_add, beside the reader's: C3 /
  // C5 at pop 1M measured no better with 1 or 4)
  const int nth = n >= 65536 ? host_threads() : 1;
  std::vector<uint8_t> too_deep((size_t)nth, 0);
  std::vector<int64_t> n_err((size_t)nth, 0), n_status((size_t)nth, 0);
  const bool asm_on = ctx->asm_ready && ctx->use_asm && ctx->nv <= 63;
  int32_t* cost = ctx->cost.data();
  int32_t* depth = ctx->depth.data();
  uint8_t* asm_ok = ctx->asm_ok.data();
  const int64_t trig_w = ctx->trig_w, div_w = ctx->div_w;
  hostpool::par_run(nth, [&](int t) {
    bool deep = false;
    int64_t ne = 0, ns = 0;
    for (int64_t i = a + n * t / nth, b = a + n * (t + 1) / nth; i < b; ++i) {
      const uint32_t m = meta[(size_t)i];
      const int32_t d = (int32_t)(m & 0xffu);
      out_depth[i] = d;
      out_err[i] = (uint8_t)((m >> 8) & 7u);
      out_status[i] = (uint8_t)((m >> 11) & 7u);
      ne += ((m >> 8) & 7u) != 0;
      ns += ((m >> 11) & 7u) != 0;
      deep |= d > kDeepDepth;
      cost[i] = (int32_t)std::min<int64_t>(nw[(size_t)i] +
                                               trig_w * (int64_t)((m >> 15) & 0xfffu) +
                                               div_w * (int64_t)(m >> 27),
                                           INT32_MAX);
      depth[i] = d;
      asm_ok[i] = core_class(((m >> 14) & 1u) && asm_on, d);
    }
    too_deep[(size_t)t] = deep;
    n_err[(size_t)t] = ne;
    n_status[(size_t)t] = ns;
  });
  for (int t = 0; t < nth; ++t) {
    ctx->lw_too_deep |= too_deep[(size_t)t] != 0;
    ctx->lw_n_err += n_err[(size_t)t];
    ctx->lw_n_status += n_status[(size_t)t];
  }
}

int lower_add(gpe_ctx* ctx, const uint8_t* codes, const int64_t* node_off, int64_t n,
              const gpe_value* evals, const int64_t* eph_off) {
  if (!ctx->lw_open) return fail(ctx, GPE_E_STATE, "gpe_lower_begin not called");
  if (n < 0 || !node_off || !eph_off || ctx->lw_added + n > ctx->lw_total_n)
    return fail(ctx, GPE_E_INVALID, "bad lowering arrays");
  const int64_t total = node_off[n], n_eval = eph_off[n];
  if (total < n || (total && !codes) || (n_eval && !evals) || node_off[0] != 0 ||
      eph_off[0] != 0)
    return fail(ctx, GPE_E_INVALID, "bad lowering offsets");
  if ((int)ctx->lw_ch.size() <= ctx->lw_k) ctx->lw_ch.emplace_back();
  const hipStream_t st = ctx->lw_stream[ctx->lw_k & 1];
  LowerChunk& C = ctx->lw_ch[(size_t)ctx->lw_k++];
  C.start = ctx->lw_added;
  C.n = n;
  ctx->lw_added += n;
  ctx->lw_nodes += total;
  if (n == 0) return 0;
  const size_t N = (size_t)std::max<int64_t>(total, 1);
  // interleaved scratch (lower_trees<true>): each wave of 64 trees gets rows
  // for its longest tree; taken unless that pads the scratch past 4x the
  // nodes (a few long trees among short ones).  The same pass writes each
  // tree's length and ephemeral count in 16 bits: those cross PCIe instead
  // of the two offset arrays, which device scans rebuild.
  const int64_t n_waves = (n + 63) / 64;
  std::vector<int64_t>& wrow = C.wrow_h;
  std::vector<int64_t>& wword = C.wword_h;
  std::vector<uint16_t>& l16 = C.l16_h;
  wrow.resize((size_t)n_waves + 1);
  wword.resize((size_t)n_waves + 1);
  l16.resize(2 * ((size_t)n + 1));
  bool wide = false;
  {
    // (threads from 2^16 trees: the evaluator's chunks are at most 2^18)
    const int nth = n >= 65536 ? host_threads() : 1;
    std::vector<uint8_t> tw((size_t)nth, 0);
    hostpool::par_run(nth, [&](int t) {
      for (int64_t w = n_waves * t / nth, e = n_waves * (t + 1) / nth; w < e; ++w) {
        int64_t m = 1;
        for (int64_t i = w * 64, ie = std::min<int64_t>(n, i + 64); i < ie; ++i) {
          const int64_t len = node_off[i + 1] - node_off[i];
          const int64_t ne = eph_off[i + 1] - eph_off[i];
          m = std::max<int64_t>(m, len);
          if (len > 0xffff || ne > 0xffff || len < 0 || ne < 0) tw[(size_t)t] = 1;
          l16[(size_t)i] = (uint16_t)len;
          l16[(size_t)n + 1 + (size_t)i] = (uint16_t)ne;
        }
        wrow[(size_t)w + 1] = m;
      }
    });
    for (uint8_t x : tw) wide |= x != 0;
    l16[(size_t)n] = 0;
    l16[2 * (size_t)n + 1] = 0;
    wrow[0] = 0;
    wword[0] = 0;
    for (int64_t w = 0; w < n_waves; ++w) {
      wword[(size_t)w + 1] = wword[(size_t)w] + 3 * wrow[(size_t)w + 1] + 1;
      wrow[(size_t)w + 1] += wrow[(size_t)w];
    }
  }
  const bool packed_off = n >= 65536 && !wide;
  const bool il = ctx->lw_interleave && 64 * wrow[(size_t)n_waves] <= 4 * (int64_t)N + 64 * 64;
  C.il = il;
  const size_t NS = il ? (size_t)64 * wrow[(size_t)n_waves] : N;
  const size_t NW = il ? (size_t)64 * wword[(size_t)n_waves] : 3 * N + (size_t)n + 1;
  if (ensure_slack(ctx, &C.codes, &C.codes_cap, N) ||
      ensure_slack(ctx, &C.node_off, &C.node_off_cap, (size_t)n + 1) ||
      ensure_slack(ctx, &C.eph_off, &C.eph_off_cap, (size_t)n + 1) ||
      ensure_slack(ctx, &C.evals, &C.evals_cap, (size_t)std::max<int64_t>(n_eval, 1)) ||
      ensure_slack(ctx, &C.rec, &C.rec_cap, NS) ||
      (ctx->machine == GPE_MACHINE_F && ensure_slack(ctx, &C.ib, &C.ib_cap, NS)) ||
      ensure_slack(ctx, &C.stk, &C.stk_cap, NS) || ensure_slack(ctx, &C.cv, &C.cv_cap, NS) ||
      ensure_slack(ctx, &C.words, &C.words_cap, NW) ||
      ensure_slack(ctx, &C.wrow, &C.wrow_cap, (size_t)n_waves + 1) ||
      ensure_slack(ctx, &C.l16, &C.l16_cap, 2 * ((size_t)n + 1)) ||
      ensure_slack(ctx, &C.wword, &C.wword_cap, (size_t)n_waves + 1))
    return GPE_E_HIP;
  {
    // through the chunk's own staging: the copies may still be in flight
    // when the next chunk is added (gpe_lower_end syncs before any reuse)
    const size_t ob = packed_off ? 0 : ((size_t)n + 1) * sizeof(int64_t);
    const HostPiece pc[7] = {
        {C.codes, codes, (size_t)total},
        {C.node_off, node_off, ob},
        {C.eph_off, eph_off, ob},
        {C.l16, l16.data(), packed_off ? l16.size() * sizeof(uint16_t) : 0},
        {C.evals, evals, (size_t)n_eval * sizeof(lowering::Val)},
        {C.wrow, wrow.data(), il ? ((size_t)n_waves + 1) * sizeof(int64_t) : 0},
        {C.wword, wword.data(), il ? ((size_t)n_waves + 1) * sizeof(int64_t) : 0}};
    if (int rc = h2d_staged_buf(ctx, &C.h_pin, &C.h_pin_cap, pc, 7, st)) return rc;
    if (packed_off) {
      // node and ephemeral offsets from the 16-bit counts
      hipcub::TransformInputIterator<int64_t, U16ToI64, const uint16_t*> ln(C.l16, U16ToI64());
      hipcub::TransformInputIterator<int64_t, U16ToI64, const uint16_t*> le(C.l16 + n + 1,
                                                                           U16ToI64());
      // (the chunk's own temporary storage: chunks run on two streams)
      size_t tmp_bytes = 0;
      HIPCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, ln, C.node_off, (int)(n + 1),
                                              st));
      if (ensure_slack(ctx, &C.scan_tmp, &C.scan_tmp_cap, tmp_bytes)) return GPE_E_HIP;
      HIPCHK(hipcub::DeviceScan::ExclusiveSum(C.scan_tmp, tmp_bytes, ln, C.node_off,
                                              (int)(n + 1), st));
      HIPCHK(hipcub::DeviceScan::ExclusiveSum(C.scan_tmp, tmp_bytes, le, C.eph_off,
                                              (int)(n + 1), st));
    }
  }
  const lowering::Tables T{ctx->d_lw_entries, ctx->d_lw_leaf, ctx->lw_n_leaf, ctx->lw_nv,
                           ctx->machine == GPE_MACHINE_F ? 0 : 1, ctx->neg_fold};
  hipLaunchKernelGGL(il ? lower_trees<true> : lower_trees<false>,
                     dim3((unsigned)((n + 127) / 128)), dim3(128), 0, st, C.codes,
                     C.node_off, C.eph_off, C.evals, T, n, C.rec, C.stk, C.cv,
                     ctx->machine == GPE_MACHINE_F ? C.ib : nullptr, C.words,
                     (const int64_t*)C.wrow, (const int64_t*)C.wword, ctx->d_lw_nw + C.start,
                     ctx->d_lw_meta + C.start);
  HIPCHK(hipGetLastError());
  // the chunk's word counts and metadata back behind it; the chunks whose
  // copies have landed are decoded here, on the caller's lowering thread
  // (read_lower: while the next chunk is read), not at gpe_lower_end
  HIPCHK(hipMemcpyAsync(ctx->lw_hm + C.start, ctx->d_lw_nw + C.start, n * sizeof(uint32_t),
                        hipMemcpyDeviceToHost, st));
  HIPCHK(hipMemcpyAsync(ctx->lw_hm + ctx->lw_total_n + C.start, ctx->d_lw_meta + C.start,
                        n * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  if (!C.ev) HIPCHK(hipEventCreateWithFlags(&C.ev, hipEventDisableTiming));
  HIPCHK(hipEventRecord(C.ev, st));
  if (ctx->lw_out_depth)
    for (; ctx->lw_dec < ctx->lw_k - 1; ++ctx->lw_dec) {
      const LowerChunk& D = ctx->lw_ch[(size_t)ctx->lw_dec];
      if (D.n) {
        const hipError_t q = hipEventQuery(D.ev);
        if (q == hipErrorNotReady) break;
        HIPCHK(q);
        decode_lowered(ctx, D.start, D.n, ctx->lw_out_depth, ctx->lw_out_err,
                       ctx->lw_out_status);
      }
    }
  return 0;
}

int lower_end(gpe_ctx* ctx, int32_t* out_depth, uint8_t* out_err, uint8_t* out_status) {
  if (!ctx->lw_open) return fail(ctx, GPE_E_STATE, "gpe_lower_begin not called");
  ctx->lw_open = false;
  const int64_t n = ctx->lw_total_n;
  if (ctx->lw_added != n) return fail(ctx, GPE_E_INVALID, "the chunks do not add up to the trees");
  if (ctx->lw_out_depth) {
    // gpe_lower_begin_into: its outputs (the same pointers, or none here)
    if ((out_depth && out_depth != ctx->lw_out_depth) || (out_err && out_err != ctx->lw_out_err) ||
        (out_status && out_status != ctx->lw_out_status))
      return fail(ctx, GPE_E_INVALID, "outputs differ from gpe_lower_begin_into's");
    out_depth = ctx->lw_out_depth;
    out_err = ctx->lw_out_err;
    out_status = ctx->lw_out_status;
  } else {
    ctx->lw_dec = 0;                 // (nothing decoded yet)
  }
  if (n > 0 && (!out_depth || !out_err || !out_status))
    return fail(ctx, GPE_E_INVALID, "bad lowering arrays");
  const auto t_l0 = std::chrono::steady_clock::now();
  auto lap = [&](const char* what) {
    if (ctx->diag)
      fprintf(stderr, "gpe_lower_end %s %.3f ms @%.3f\n", what,
              std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_l0)
                  .count(), diag_stamp());
  };
  const size_t N = (size_t)std::max<int64_t>(ctx->lw_nodes, 1);
  // the programs' words are compacted on the device before their count
  // reaches the host: room for the most they can take (3 per node + END)
  if (ensure(ctx, &ctx->d_code, &ctx->code_cap, 3 * N + (size_t)n + 1 + kCodePad))
    return GPE_E_HIP;
  for (int c = 0; c < ctx->lw_k; ++c)      // every chunk's lowering, on its stream
    if (ctx->lw_ch[(size_t)c].n) HIPCHK(hipStreamWaitEvent(ctx->stream, ctx->lw_ch[(size_t)c].ev, 0));
  if (n) {
    // the offsets (a scan of the word counts) and the compaction run on the
    // device while the host decodes the chunks not decoded yet
    hipcub::TransformInputIterator<int64_t, U32ToI64, const uint32_t*> nw64(ctx->d_lw_nw,
                                                                            U32ToI64());
    size_t tmp_bytes = 0;
    HIPCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, nw64, ctx->d_off, (int)(n + 1),
                                            ctx->stream));
    if (tmp_bytes > ctx->sort_tmp_cap) {
      HIPCHK(hipStreamSynchronize(ctx->stream));
      if (ensure(ctx, &ctx->d_sort_tmp, &ctx->sort_tmp_cap, tmp_bytes)) return GPE_E_HIP;
    }
    HIPCHK(hipcub::DeviceScan::ExclusiveSum(ctx->d_sort_tmp, tmp_bytes, nw64, ctx->d_off,
                                            (int)(n + 1), ctx->stream));
    for (int c = 0; c < ctx->lw_k; ++c) {
      const LowerChunk& C = ctx->lw_ch[(size_t)c];
      if (!C.n) continue;
      hipLaunchKernelGGL(C.il ? compact_words<true> : compact_words<false>,
                         dim3((unsigned)((C.n + 255) / 256)), dim3(256), 0, ctx->stream,
                         C.words, C.node_off, (const int64_t*)C.wword, ctx->d_off + C.start,
                         C.n, ctx->d_code);
      HIPCHK(hipGetLastError());
    }
    static_assert(kCodePad <= 1024, "pad_code: one block");
    hipLaunchKernelGGL(pad_code, dim3(1), dim3(kCodePad), 0, ctx->stream, ctx->d_code,
                       (const int64_t*)ctx->d_off, n, (int)kCodePad);
    HIPCHK(hipGetLastError());
    // the remaining chunks, as their metadata lands (each chunk's event)
    int first = ctx->lw_dec;
    for (int c = first; c < ctx->lw_k; ++c) {
      const LowerChunk& C = ctx->lw_ch[(size_t)c];
      if (!C.n) continue;
      HIPCHK(hipEventSynchronize(C.ev));
      if (c == first) lap("metadata");
      decode_lowered(ctx, C.start, C.n, out_depth, out_err, out_status);
    }
    ctx->lw_dec = ctx->lw_k;
  } else {
    HIPCHK(hipMemsetAsync(ctx->d_off, 0, sizeof(int64_t), ctx->stream));
    HIPCHK(hipMemsetAsync(ctx->d_code, 0, kCodePad * sizeof(uint32_t), ctx->stream));
  }
  ctx->lw_out_depth = nullptr;
  ctx->lw_out_err = nullptr;
  ctx->lw_out_status = nullptr;
  if (ctx->lw_too_deep) return fail(ctx, GPE_E_DEPTH, "program needs more than 32 stack slots");
  lap("host pass");
  ctx->n_prog = n;
  ctx->acode_prec = -1;
  ctx->typed_valid = false;
  // (threaded code: translated on the device by the first run that needs it)
  ctx->planned_mode = -1;
  if (ensure(ctx, &ctx->d_hi, &ctx->hi_cap, (size_t)n)) return GPE_E_HIP;
  if (ensure(ctx, &ctx->d_lo, &ctx->lo_cap, (size_t)n)) return GPE_E_HIP;
  if (ensure(ctx, &ctx->d_err, &ctx->err_cap, (size_t)n)) return GPE_E_HIP;
  if (ensure(ctx, &ctx->d_flags, &ctx->flags_cap, (size_t)n)) return GPE_E_HIP;
  HIPCHK(hipStreamSynchronize(ctx->stream));
  lap("done");
  return 0;
}

}  // namespace

extern "C" {

int gpe_lower_begin(gpe_ctx* ctx, int64_t n_total) {
  if (!ctx) return GPE_E_INVALID;
  ctx->lw_open = false;
  ctx->last_mode = -1;         // resident fitness no longer matches
  ctx->n_exact = 0;            // the exact pass belongs to a population
  ctx->ex_all = 0;
  if (ctx->machine < 0) return fail(ctx, GPE_E_STATE, "gpe_set_cases not called");
  if (ctx->lw_machine != ctx->machine)
    return fail(ctx, GPE_E_STATE, "gpe_set_lowering not called for this machine");
  if (n_total < 0 || n_total > INT32_MAX) return fail(ctx, GPE_E_INVALID, "bad tree count");
  HIPCHK(hipSetDevice(ctx->device));
  // an abandoned lowering (read_lower declined a chunk, or gpe_lower_add
  // failed) may have chunks in flight on the lowering queues: their
  // uploads, kernels and metadata copies read the pinned staging and write
  // d_lw_nw / d_lw_meta / lw_hm, all rewritten below — drain both queues
  // (ctx->stream alone does not order them)
  for (hipStream_t st : ctx->lw_stream)
    if (st) HIPCHK(hipStreamSynchronize(st));
  // the program buffers are rewritten from here on: a failed lowering leaves
  // the context without programs, not with a mix
  ctx->n_prog = 0;
  ctx->planned_mode = -1;
  if (ensure(ctx, &ctx->d_lw_nw, &ctx->lw_nw_cap, (size_t)n_total + 1) ||
      ensure(ctx, &ctx->d_lw_meta, &ctx->lw_meta_cap, (size_t)std::max<int64_t>(n_total, 1)) ||
      ensure(ctx, &ctx->d_off, &ctx->off_cap, (size_t)n_total + 1))
    return GPE_E_HIP;
  const size_t hm_bytes = 2 * (size_t)std::max<int64_t>(n_total, 1) * sizeof(uint32_t);
  if (hm_bytes > ctx->lw_hm_cap)     // (a failed lowering's copies may be in flight)
    HIPCHK(hipStreamSynchronize(ctx->stream));
  if (!pinned_buf((char**)&ctx->lw_hm, &ctx->lw_hm_cap, hm_bytes))
    return fail(ctx, GPE_E_HIP, "hipHostMalloc (lowering metadata)");
  HIPCHK(hipMemsetAsync(ctx->d_lw_nw + n_total, 0, sizeof(uint32_t), ctx->stream));
  for (hipStream_t& st : ctx->lw_stream) {
    if (!st) HIPCHK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  }
  HIPCHK(hipEventRecord(ctx->ev_lw, ctx->stream));
  for (hipStream_t st : ctx->lw_stream) HIPCHK(hipStreamWaitEvent(st, ctx->ev_lw, 0));
  // the per-program vectors, written chunk by chunk (resized, not refilled:
  // every entry is written)
  ctx->cost.resize((size_t)n_total);
  ctx->depth.resize((size_t)n_total);
  ctx->asm_ok.resize((size_t)n_total);
  ctx->lw_out_depth = nullptr;
  ctx->lw_out_err = nullptr;
  ctx->lw_out_status = nullptr;
  ctx->lw_dec = 0;
  ctx->lw_too_deep = false;
  ctx->lw_n_err = ctx->lw_n_status = 0;
  ctx->lw_k = 0;
  ctx->lw_total_n = n_total;
  ctx->lw_added = 0;
  ctx->lw_nodes = 0;
  ctx->lw_open = true;
  return 0;
}

int gpe_lower_begin_into(gpe_ctx* ctx, int64_t n_total, int32_t* out_depth, uint8_t* out_err,
                         uint8_t* out_status) {
  if (!ctx) return GPE_E_INVALID;
  if (n_total > 0 && (!out_depth || !out_err || !out_status))
    return fail(ctx, GPE_E_INVALID, "bad lowering arrays");
  const int rc = gpe_lower_begin(ctx, n_total);
  if (rc) return rc;
  if (n_total > 0) {
    ctx->lw_out_depth = out_depth;
    ctx->lw_out_err = out_err;
    ctx->lw_out_status = out_status;
  }
  return 0;
}

int gpe_lower_add(gpe_ctx* ctx, const uint8_t* codes, const int64_t* node_off, int64_t n,
                  const gpe_value* evals, const int64_t* eph_off) {
  if (!ctx) return GPE_E_INVALID;
  HIPCHK(hipSetDevice(ctx->device));
  const auto t0 = std::chrono::steady_clock::now();
  const int rc = lower_add(ctx, codes, node_off, n, evals, eph_off);
  if (ctx->diag)
    fprintf(stderr, "gpe_lower_add %lld trees @%.3f %.3f ms\n", (long long)n, diag_stamp(),
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0)
                .count());
  if (rc) ctx->lw_open = false;
  return rc;
}

int gpe_lower_end(gpe_ctx* ctx, int32_t* out_depth, uint8_t* out_err, uint8_t* out_status) {
  if (!ctx) return GPE_E_INVALID;
  HIPCHK(hipSetDevice(ctx->device));
  return lower_end(ctx, out_depth, out_err, out_status);
}

int gpe_lower_programs(gpe_ctx* ctx, const uint8_t* codes, const int64_t* node_off,
                       int64_t n, const gpe_value* evals, const int64_t* eph_off,
                       int32_t* out_depth, uint8_t* out_err, uint8_t* out_status) {
  if (!ctx) return GPE_E_INVALID;
  if (n < 0 || !node_off || !eph_off || !out_depth || !out_err || !out_status)
    return fail(ctx, GPE_E_INVALID, "bad lowering arrays");
  int rc = gpe_lower_begin(ctx, n);
  if (!rc) rc = gpe_lower_add(ctx, codes, node_off, n, evals, eph_off);
  if (!rc) rc = gpe_lower_end(ctx, out_depth, out_err, out_status);
  return rc;
}

int gpe_load_programs(gpe_ctx* ctx, const uint32_t* code, int64_t n_words,
                      const int64_t* off, int64_t n_prog,
                      const int32_t* depth) {
  if (!ctx) return GPE_E_INVALID;
  ctx->last_mode = -1;         // resident fitness no longer matches
  ctx->n_exact = 0;            // the exact pass belongs to a population
  ctx->ex_all = 0;
  if (ctx->machine < 0) return fail(ctx, GPE_E_STATE, "gpe_set_cases not called");
  if (n_prog < 0 || n_words < 0 || (n_prog > 0 && (!code || !off || !depth)))
    return fail(ctx, GPE_E_INVALID, "bad program arrays");
  if (n_prog > INT32_MAX) return fail(ctx, GPE_E_INVALID, "too many programs");
  HIPCHK(hipSetDevice(ctx->device));
  const auto t_l0 = std::chrono::steady_clock::now();
  auto lap = [&](const char* what) {
    if (ctx->diag)
      fprintf(stderr, "gpe_load_programs %s %.3f ms\n", what,
              std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_l0)
                  .count());
  };
  ctx->cost.assign((size_t)n_prog, 0);
  ctx->depth.assign(depth, depth + n_prog);
  ctx->asm_ok.assign((size_t)n_prog, 0);
  // validation in host threads (contiguous program ranges); the first
  // failing program in index order is reported
  const int nth = (int)std::max<int64_t>(1, std::min<int64_t>(host_threads(), n_prog / 8192));
  std::vector<int64_t> bad_at((size_t)nth, -1);
  std::vector<std::string> bad_why((size_t)nth);
  std::vector<int> bad_code((size_t)nth, 0);
  auto check = [&](int t) {
    const int64_t a = n_prog * t / nth, b = n_prog * (t + 1) / nth;
    for (int64_t i = a; i < b; ++i) {
      if (off[i] < 0 || off[i + 1] > n_words || off[i + 1] <= off[i]) {
        bad_at[t] = i;
        bad_code[t] = GPE_E_INVALID;
        bad_why[t] = "program offsets out of range";
        return;
      }
      bool ok = false;
      int64_t n_trig = 0, n_div = 0;
      std::string why = validate_program(code + off[i], off[i + 1] - off[i],
                                         ctx->machine, ctx->nv, depth[i], &ok,
                                         &n_trig, &n_div);
      if (!why.empty()) {
        bad_at[t] = i;
        bad_code[t] = GPE_E_INVALID;
        bad_why[t] = "program " + std::to_string(i) + ": " + why;
        return;
      }
      if (depth[i] > kDeepDepth) {
        bad_at[t] = i;
        bad_code[t] = GPE_E_DEPTH;
        bad_why[t] = "program needs more than 32 stack slots";
        return;
      }
      ctx->cost[(size_t)i] =
          (int32_t)std::min<int64_t>(off[i + 1] - off[i] + ctx->trig_w * n_trig +
                                         ctx->div_w * n_div, INT32_MAX);
      ctx->asm_ok[(size_t)i] =
          core_class(ok && ctx->asm_ready && ctx->use_asm && ctx->nv <= 63, depth[i]);
    }
  };
  if (nth == 1) {
    check(0);
  } else {
    hostpool::par_run(nth, check);
  }
  for (int t = 0; t < nth; ++t)
    if (bad_at[t] >= 0) return fail(ctx, bad_code[t], bad_why[t]);
  lap("validated");
  if (ensure(ctx, &ctx->d_code, &ctx->code_cap, (size_t)n_words + kCodePad))
    return GPE_E_HIP;
  HIPCHK(hipMemsetAsync(ctx->d_code + n_words, 0, kCodePad * sizeof(uint32_t),
                        ctx->stream));                       // OP_END pad
  if (ensure(ctx, &ctx->d_off, &ctx->off_cap, (size_t)n_prog + 1)) return GPE_E_HIP;
  {
    const HostPiece pc[2] = {{ctx->d_code, code, (size_t)n_words * sizeof(uint32_t)},
                             {ctx->d_off, off, ((size_t)n_prog + 1) * sizeof(int64_t)}};
    if (int rc = h2d_staged(ctx, pc, 2)) return rc;
  }
  lap("staged");
  ctx->n_prog = n_prog;
  // threaded code for the asm core of the current precision: translated by
  // plan_mode for the first MSE run (again if the precision changes)
  ctx->acode_prec = -1;
  ctx->typed_valid = false;

  ctx->planned_mode = -1;
  if (ensure(ctx, &ctx->d_hi, &ctx->hi_cap, (size_t)n_prog)) return GPE_E_HIP;
  if (ensure(ctx, &ctx->d_lo, &ctx->lo_cap, (size_t)n_prog)) return GPE_E_HIP;
  if (ensure(ctx, &ctx->d_err, &ctx->err_cap, (size_t)n_prog)) return GPE_E_HIP;
  if (ensure(ctx, &ctx->d_flags, &ctx->flags_cap, (size_t)n_prog)) return GPE_E_HIP;
  HIPCHK(hipStreamSynchronize(ctx->stream));
  lap("done");
  return 0;
}

namespace {
// GPE_MODE_SSE_NUMPY: the MSE-mode run writes every squared term to the
// per-case matrix, then np_sum_rows reduces each row in numpy's order.
int run_numpy(gpe_ctx* ctx, int mode, double* hi, double* lo,
              unsigned long long* err, uint32_t* flags) {
  if (ctx->machine != GPE_MACHINE_F || ctx->nt < 1)
    return fail(ctx, GPE_E_INVALID, "row-sum modes need the F machine and a target");
  if (ctx->n_prog <= 0) return run_common(ctx, GPE_MODE_MSE, hi, lo, err, flags);
  const size_t n = (size_t)ctx->n_prog * (size_t)ctx->n_cases;
  if (ensure(ctx, &ctx->d_case_out, &ctx->case_cap, n)) return GPE_E_HIP;
  if (mode == GPE_MODE_SSE_SEQ) {
    ctx->case_on = 1;
    int rc = run_common(ctx, GPE_MODE_MSE, hi, lo, err, flags);
    ctx->case_on = 0;
    if (rc) return rc;
    hipLaunchKernelGGL(seq_sum_rows, dim3((unsigned)((ctx->n_prog + 255) / 256)),
                       dim3(256), 0, ctx->stream, ctx->d_case_out, ctx->n_cases,
                       ctx->n_prog, hi, lo);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(ctx->stream));
    return 0;
  }
  if (ctx->np_n != ctx->n_cases) {
    const NpPlan p = np_plan(ctx->n_cases);
    if (p.depth > kNpStack) return fail(ctx, GPE_E_INVALID, "numpy plan too deep");
    for (void* b : {(void*)ctx->d_np_off, (void*)ctx->d_np_len, (void*)ctx->d_np_post})
      if (b) HIPCHK(hipFree(b));
    ctx->d_np_off = nullptr;
    ctx->d_np_len = ctx->d_np_post = nullptr;
    ctx->np_n = 0;
    HIPCHK(hipMalloc(&ctx->d_np_off, p.off.size() * sizeof(int64_t)));
    HIPCHK(hipMalloc(&ctx->d_np_len, p.len.size() * sizeof(int32_t)));
    HIPCHK(hipMalloc(&ctx->d_np_post, p.post.size() * sizeof(int32_t)));
    HIPCHK(hipMemcpy(ctx->d_np_off, p.off.data(), p.off.size() * sizeof(int64_t), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(ctx->d_np_len, p.len.data(), p.len.size() * sizeof(int32_t), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(ctx->d_np_post, p.post.data(), p.post.size() * sizeof(int32_t), hipMemcpyHostToDevice));
    ctx->np_leaves = (int)p.off.size();
    ctx->np_post = (int)p.post.size();
    ctx->np_n = ctx->n_cases;
  }
  if (ensure(ctx, &ctx->d_np_leaf, &ctx->np_leaf_cap,
             (size_t)ctx->n_prog * (size_t)ctx->np_leaves)) return GPE_E_HIP;
  ctx->case_on = 1;
  int rc = run_common(ctx, GPE_MODE_MSE, hi, lo, err, flags);
  ctx->case_on = 0;
  if (rc) return rc;
  hipLaunchKernelGGL(np_sum_rows, dim3((unsigned)ctx->n_prog), dim3(64), 0, ctx->stream,
                     ctx->d_case_out, ctx->n_cases, ctx->d_np_off, ctx->d_np_len,
                     ctx->np_leaves, ctx->d_np_post, ctx->np_post, ctx->d_np_leaf, hi, lo);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(ctx->stream));
  return 0;
}

int run_mode(gpe_ctx* ctx, int mode, double* hi, double* lo,
             unsigned long long* err, uint32_t* flags) {
  if (mode == GPE_MODE_SSE_NUMPY || mode == GPE_MODE_SSE_SEQ)
    return run_numpy(ctx, mode, hi, lo, err, flags);
  return run_common(ctx, mode, hi, lo, err, flags);
}

// The context's own output buffers now hold the fitness of the loaded
// programs on the loaded cases: gpe_tournament(NULL, ...) may select on them.
void keep_resident(gpe_ctx* ctx, int mode, bool sharded) {
  ctx->last_mode = mode;
  ctx->last_n = ctx->n_prog;
  ctx->last_cases = (double)ctx->n_cases;
  ctx->last_cases_dev = sharded;
}
}  // namespace

int gpe_set_precision(gpe_ctx* ctx, int prec) {
  if (!ctx) return GPE_E_INVALID;
  if (prec != GPE_PREC_F64 && prec != GPE_PREC_F32)
    return fail(ctx, GPE_E_INVALID, "precision must be GPE_PREC_F64 or GPE_PREC_F32");
  if (prec != ctx->prec) ctx->planned_mode = -1;
  ctx->prec = prec;
  return 0;
}

int gpe_run_device(gpe_ctx* ctx, int mode, void* d_hi, void* d_lo,
                   void* d_err, void* d_flags) {
  if (!ctx) return GPE_E_INVALID;
  HIPCHK(hipSetDevice(ctx->device));
  const int rc = run_mode(ctx, mode, d_hi ? (double*)d_hi : ctx->d_hi,
                          d_lo ? (double*)d_lo : ctx->d_lo,
                          d_err ? (unsigned long long*)d_err : ctx->d_err,
                          d_flags ? (uint32_t*)d_flags : ctx->d_flags);
  // caller-owned outputs are never read back by gpe_tournament
  if (!rc && !d_hi && !d_lo && !d_err && !d_flags) keep_resident(ctx, mode, false);
  return rc;
}

// The resident results (d_hi/d_lo/d_err/d_flags) into the caller's arrays:
// device -> pinned staging -> host threads.  (A synchronous copy into
// pageable arrays lets the runtime pin them in place; when Python later frees
// them, the next stream operation stalled 10-30 ms on the box at pop 1M.)
int results_to_host(gpe_ctx* ctx, size_t n, double* out_hi, double* out_lo, uint64_t* out_err,
                    uint32_t* out_flags) {
  if (!n) return 0;
  struct Piece { void* dst; const void* src; size_t bytes; size_t at; };
  Piece pc[4] = {{out_hi, ctx->d_hi, n * sizeof(double), 0},
                 {out_lo, ctx->d_lo, n * sizeof(double), 0},
                 {out_err, ctx->d_err, n * sizeof(uint64_t), 0},
                 {out_flags, ctx->d_flags, n * sizeof(uint32_t), 0}};
  size_t total = 0;
  for (Piece& p : pc) {
    p.at = total;
    if (p.dst) total += (p.bytes + 63) / 64 * 64;
  }
  if (!total) return 0;
  char* stage = pinned_buf(&ctx->h_pin_in, &ctx->h_pin_in_cap, total);
  if (!stage) return fail(ctx, GPE_E_HIP, "hipHostMalloc (results)");
  for (const Piece& p : pc)
    if (p.dst)
      HIPCHK(hipMemcpyAsync(stage + p.at, p.src, p.bytes, hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  const int nth = total >= ((size_t)4 << 20) ? host_threads() : 1;
  auto copy = [&](int t) {
    for (const Piece& p : pc) {
      if (!p.dst) continue;
      const size_t a = p.bytes * t / nth, b = p.bytes * (t + 1) / nth;
      if (b > a) std::memcpy((char*)p.dst + a, stage + p.at + a, b - a);
    }
  };
  if (nth == 1) {
    copy(0);
  } else {
    hostpool::par_run(nth, copy);
  }
  return 0;
}

int gpe_run(gpe_ctx* ctx, int mode, double* out_hi, double* out_lo,
            uint64_t* out_err, uint32_t* out_flags) {
  if (!ctx) return GPE_E_INVALID;
  HIPCHK(hipSetDevice(ctx->device));
  const auto t_r0 = std::chrono::steady_clock::now();
  int rc = run_mode(ctx, mode, ctx->d_hi, ctx->d_lo, ctx->d_err, ctx->d_flags);
  if (rc) return rc;
  keep_resident(ctx, mode, false);
  const auto t_r1 = std::chrono::steady_clock::now();
  const size_t n = (size_t)ctx->n_prog;
  if (int rc_d = results_to_host(ctx, n, out_hi, out_lo, out_err, out_flags)) return rc_d;
  if (ctx->diag) {
    const auto t_r2 = std::chrono::steady_clock::now();
    fprintf(stderr, "gpe_run run %.3f ms, d2h %.3f ms\n",
            std::chrono::duration<double, std::milli>(t_r1 - t_r0).count(),
            std::chrono::duration<double, std::milli>(t_r2 - t_r1).count());
  }
  return 0;
}

int gpe_run_cases(gpe_ctx* ctx, int mode, double* out_cases, double* out_hi,
                  double* out_lo, uint64_t* out_err, uint32_t* out_flags) {
  if (!ctx || !out_cases) return GPE_E_INVALID;
  if (ctx->machine != GPE_MACHINE_F || mode == GPE_MODE_HITS_BITS)
    return fail(ctx, GPE_E_INVALID, "per-case output needs the F machine");
  HIPCHK(hipSetDevice(ctx->device));
  const size_t n = (size_t)ctx->n_prog * (size_t)ctx->n_cases;
  if (ensure(ctx, &ctx->d_case_out, &ctx->case_cap, n)) return GPE_E_HIP;
  ctx->case_on = 1;
  int rc = run_common(ctx, mode, ctx->d_hi, ctx->d_lo, ctx->d_err, ctx->d_flags);
  ctx->case_on = 0;
  if (rc) return rc;
  keep_resident(ctx, mode, false);
  HIPCHK(hipMemcpy(out_cases, ctx->d_case_out, n * sizeof(double), hipMemcpyDeviceToHost));
  const size_t np = (size_t)ctx->n_prog;
  if (int rc_d = results_to_host(ctx, np, out_hi, out_lo, out_err, out_flags)) return rc_d;
  return 0;
}

int gpe_eval(gpe_ctx* ctx, int mode, const uint32_t* code, int64_t n_words,
             const int64_t* off, int64_t n_prog, const int32_t* depth,
             double* out_hi, double* out_lo, uint64_t* out_err,
             uint32_t* out_flags) {
  int rc = gpe_load_programs(ctx, code, n_words, off, n_prog, depth);
  if (rc) return rc;
  return gpe_run(ctx, mode, out_hi, out_lo, out_err, out_flags);
}

int gpe_load_exact_v(gpe_ctx* ctx, const int32_t* progs, int64_t n, const uint32_t* code,
                     int64_t n_words, const int64_t* off, const int32_t* depth,
                     const uint32_t* int_words, const int64_t* int_off, int64_t n_ints) {
  if (!ctx || n < 0 || n_ints < 0 || n_words < 0) return GPE_E_INVALID;
  HIPCHK(hipSetDevice(ctx->device));
  ctx->n_exact = 0;
  ctx->ex_all = 0;
  ctx->last_mode = -1;
  if (n == 0) return 0;
  if (!progs || !code || !off || !depth || (n_ints && (!int_words || !int_off)))
    return GPE_E_INVALID;
  if (ctx->machine != GPE_MACHINE_F)
    return fail(ctx, GPE_E_INVALID, "the exact pass runs F-machine programs");
  if (off[0] != 0 || off[n] != n_words)
    return fail(ctx, GPE_E_INVALID, "exact programs: offsets do not span the words");
  if (n_ints && int_off[0] != 0)
    return fail(ctx, GPE_E_INVALID, "exact programs: int rows must start at word 0");
  for (int64_t r = 0; r < n_ints; ++r)
    if (int_off[r + 1] < int_off[r])
      return fail(ctx, GPE_E_INVALID, "exact programs: bad int row offsets");
  // a row the device holds: a value of 1088-bit two's complement (the words
  // past kWords only extend the sign)
  std::vector<uint8_t> narrow((size_t)n_ints, 1);
  std::vector<uint32_t> dev_ints((size_t)std::max<int64_t>(n_ints, 1) * xint::kWords, 0);
  for (int64_t r = 0; r < n_ints; ++r) {
    const uint32_t* w = int_words + int_off[r];
    const int64_t len = int_off[r + 1] - int_off[r];
    const uint32_t ext = (len && (w[len - 1] >> 31)) ? 0xffffffffu : 0u;
    bool fits = true;
    for (int64_t k = xint::kWords; k < len; ++k) fits &= w[k] == ext;
    if (len >= xint::kWords) fits &= (w[xint::kWords - 1] >> 31) == (ext & 1u);
    narrow[(size_t)r] = fits;
    for (int k = 0; k < xint::kWords; ++k)
      dev_ints[(size_t)r * xint::kWords + k] = k < len ? w[k] : ext;
  }
  std::vector<int32_t> dprogs;
  std::vector<uint32_t> dcode;
  std::vector<int64_t> doff{0}, dev_index, host;
  for (int64_t i = 0; i < n; ++i) {
    if (progs[i] < 0 || progs[i] >= ctx->n_prog)
      return fail(ctx, GPE_E_INVALID, "exact programs: program index out of range");
    if (off[i + 1] < off[i] || depth[i] < 0 || depth[i] > kXintDepth)
      return fail(ctx, GPE_E_INVALID, "exact programs: bad offsets or depth beyond 32");
    const uint32_t* w = code + off[i];
    const int64_t len = off[i + 1] - off[i];
    bool asm_ok = false;
    std::string e = validate_program(w, len, GPE_MACHINE_F, ctx->nv, depth[i], &asm_ok);
    if (!e.empty()) return fail(ctx, GPE_E_INVALID, "exact program " + std::to_string(i) + ": " + e);
    bool dev = true;
    for (int64_t k = 0; k < len; ++k) {     // opcodes and int constant rows
      const uint32_t op = w[k] & 0xffu, tag = w[k] >> 16;
      if (op >= OP_NPDIV || op == OP_XOR || op == OP_XOR + 1 || op == OP_XOR + 2)
        return fail(ctx, GPE_E_INVALID, "exact programs: numpy / xor opcode");
      const bool konst = op == OP_LDC || op == OP_PUSHC ||
                         (op >= OP_ADD && op < OP_NEG && (op - OP_ADD) % 3 == 2);
      if (konst) {
        if (k + 2 >= len) return fail(ctx, GPE_E_INVALID, "exact programs: truncated constant");
        if (tag) {
          const uint64_t r = (uint64_t)w[k + 1] | ((uint64_t)w[k + 2] << 32);
          if (tag != 1 || r >= (uint64_t)n_ints)
            return fail(ctx, GPE_E_INVALID, "exact programs: int constant row out of range");
          dev &= narrow[(size_t)r] != 0;
        }
        k += 2;
      }
    }
    if (dev) {
      dev_index.push_back(i);
      dprogs.push_back(progs[i]);
      dcode.insert(dcode.end(), w, w + len);
      doff.push_back((int64_t)dcode.size());
    } else {
      host.push_back(i);
    }
  }
  const int64_t nd = (int64_t)dprogs.size();
  if (nd) {
    if (ensure(ctx, &ctx->d_ex_progs, &ctx->ex_progs_cap, (size_t)nd) ||
        ensure(ctx, &ctx->d_ex_code, &ctx->ex_code_cap, dcode.size()) ||
        ensure(ctx, &ctx->d_ex_off, &ctx->ex_off_cap, (size_t)nd + 1) ||
        ensure(ctx, &ctx->d_ex_ints, &ctx->ex_ints_cap, dev_ints.size()))
      return GPE_E_HIP;
    HIPCHK(hipMemcpy(ctx->d_ex_progs, dprogs.data(), nd * sizeof(int32_t), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(ctx->d_ex_code, dcode.data(), dcode.size() * sizeof(uint32_t),
                     hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(ctx->d_ex_off, doff.data(), (nd + 1) * sizeof(int64_t), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(ctx->d_ex_ints, dev_ints.data(), dev_ints.size() * sizeof(uint32_t),
                     hipMemcpyHostToDevice));
  }
  ctx->ex_h_progs.assign(progs, progs + n);
  ctx->ex_h_code.assign(code, code + n_words);
  ctx->ex_h_off.assign(off, off + n + 1);
  ctx->ex_h_woff.assign(int_off, int_off + (n_ints ? n_ints + 1 : 0));
  ctx->ex_h_words.assign(int_words, int_words + (n_ints ? int_off[n_ints] : 0));
  ctx->ex_dev_index = std::move(dev_index);
  ctx->ex_host = std::move(host);
  ctx->n_exact = nd;
  ctx->ex_all = n;
  return 0;
}

int gpe_load_exact(gpe_ctx* ctx, const int32_t* progs, int64_t n, const uint32_t* code,
                   int64_t n_words, const int64_t* off, const int32_t* depth,
                   const uint32_t* ints, int64_t n_ints) {
  if (n_ints < 0 || n < 0 || n_words < 0 || (n && (!code || !off))) return GPE_E_INVALID;
  std::vector<int64_t> woff((size_t)n_ints + 1);
  for (int64_t r = 0; r <= n_ints; ++r) woff[(size_t)r] = r * xint::kWords;
  // the round-4 encoding of an int constant: index field 1 + row, the f64
  // bits in its two data words; gpe_load_exact_v's: index field 1, the row
  // in the data words (no 65,535-row cap).  Translated here, so callers of
  // this entry point keep working
  std::vector<uint32_t> cv(code, code + n_words);
  for (int64_t i = 0; i < n; ++i) {
    for (int64_t k = off[i]; k >= 0 && k < n_words; ++k) {
      const uint32_t op = cv[(size_t)k] & 0xffu;
      if (op == OP_END) break;
      const bool konst = op == OP_LDC || op == OP_PUSHC ||
                         (op >= OP_ADD && op < OP_NEG && (op - OP_ADD) % 3 == 2);
      if (!konst) continue;
      if (k + 2 >= n_words) return fail(ctx, GPE_E_INVALID, "constant past the code");
      const uint32_t t = cv[(size_t)k] >> 16;
      if (t) {
        if ((int64_t)(t - 1) >= n_ints) return fail(ctx, GPE_E_INVALID, "int constant row out of range");
        cv[(size_t)k] = (cv[(size_t)k] & 0xffffu) | (1u << 16);
        cv[(size_t)k + 1] = t - 1;
        cv[(size_t)k + 2] = 0;
      }
      k += 2;
    }
  }
  return gpe_load_exact_v(ctx, progs, n, cv.data(), n_words, off, depth, ints, woff.data(), n_ints);
}

int gpe_host_exact_eval(const uint32_t* code, const uint32_t* int_words, const int64_t* int_off,
                        int64_t n_ints, const double* x, int nv, double* out_f,
                        uint32_t* out_words, int* out_isint) {
  if (!code || !x || nv < 0 || n_ints < 0 || (n_ints && (!int_words || !int_off)))
    return GPE_E_INVALID;
  // the device's table: rows as 1088-bit two's complement; a program
  // reading a wider row is past the pass's range before it starts
  std::vector<uint32_t> tab((size_t)std::max<int64_t>(n_ints, 1) * xint::kWords, 0);
  std::vector<uint8_t> wide((size_t)std::max<int64_t>(n_ints, 1), 0);
  for (int64_t r = 0; r < n_ints; ++r) {
    const uint32_t* w = int_words + int_off[r];
    const int64_t len = int_off[r + 1] - int_off[r];
    const uint32_t ext = (len && (w[len - 1] >> 31)) ? 0xffffffffu : 0u;
    for (int64_t k = xint::kWords; k < len; ++k) wide[(size_t)r] |= w[k] != ext;
    if (len >= xint::kWords) wide[(size_t)r] |= (w[xint::kWords - 1] >> 31) != (ext & 1u);
    for (int k = 0; k < xint::kWords; ++k) tab[(size_t)r * xint::kWords + k] = k < len ? w[k] : ext;
  }
  for (int64_t k = 0;; ++k) {             // int rows the program reads
    const uint32_t op = code[k] & 0xffu;
    if (op == OP_END) break;
    const bool konst = op == OP_LDC || op == OP_PUSHC ||
                       (op >= OP_ADD && op < OP_NEG && (op - OP_ADD) % 3 == 2);
    if (!konst) continue;
    if (code[k] >> 16) {
      const uint64_t r = (uint64_t)code[k + 1] | ((uint64_t)code[k + 2] << 32);
      if (r >= (uint64_t)n_ints) return GPE_E_INVALID;
      if (wide[(size_t)r]) return (int)xint::E_RANGE;
    }
    k += 2;
  }
  xint::Num T;
  uint32_t err = xint::E_NONE;
  auto xv = [&](uint32_t v) { return (int)v < nv ? x[v] : 0.0; };
  if (!xint::run<kXintDepth>(code, tab.data(), xv, T, err)) return GPE_E_INVALID;
  if (err) return (int)err;
  if (out_isint) *out_isint = T.isint ? 1 : 0;
  uint32_t ferr = xint::E_NONE;           // float(result) (an int may overflow)
  if (out_f) *out_f = xint::to_f(T, ferr);
  if (out_words) {                         // GPE_XINT_WORDS-word two's complement
    uint64_t m[xint::kLimbs];
    for (int i = 0; i < xint::kLimbs; ++i) m[i] = T.m.w[i];
    if (T.isint && T.neg) {
      uint64_t c = 1;
      for (int i = 0; i < xint::kLimbs; ++i) {
        m[i] = ~m[i] + c;
        c = c && m[i] == 0;
      }
    }
    for (int i = 0; i < xint::kLimbs; ++i) {
      out_words[2 * i] = (uint32_t)m[i];
      out_words[2 * i + 1] = (uint32_t)(m[i] >> 32);
    }
  }
  return 0;
}

int gpe_host_bigint_eval(const uint32_t* code, const uint32_t* int_words, const int64_t* int_off,
                         int64_t n_ints, const double* x, int nv, double* out_f,
                         uint32_t* out_words, int64_t* inout_nwords, int* out_isint) {
  if (!code || !x || nv < 0 || n_ints < 0 || (n_ints && (!int_words || !int_off)))
    return GPE_E_INVALID;
  const hbig::Rows rows{int_words, int_off, n_ints};
  hbig::Num T;
  uint32_t err = hbig::E_NONE;
  auto xv = [&](uint32_t v) { return (int)v < nv ? x[v] : 0.0; };
  try {
    if (!hbig::run(code, rows, xv, T, err)) return GPE_E_INVALID;
  } catch (const std::bad_alloc&) {
    return GPE_E_INVALID;
  }
  if (err) return (int)err;
  if (out_isint) *out_isint = T.isint ? 1 : 0;
  uint32_t ferr = hbig::E_NONE;
  if (out_f) *out_f = hbig::to_f(T, ferr);
  if (inout_nwords) {                      // two's complement, one sign bit to spare
    const int64_t need = T.isint ? hbig::bitlen(T.m) / 32 + 1 : 1;
    if (!out_words || *inout_nwords < need) {
      *inout_nwords = need;
      return out_words ? GPE_E_INVALID : 0;
    }
    *inout_nwords = need;
    std::vector<uint64_t> m(T.isint ? T.m : hbig::Mag());
    m.resize((size_t)((need + 1) / 2), 0);
    if (T.isint && T.neg) {
      uint64_t c = 1;
      for (auto& v : m) {
        v = ~v + c;
        c = c && v == 0;
      }
    }
    for (int64_t i = 0; i < need; ++i) out_words[i] = (uint32_t)(m[(size_t)(i / 2)] >> (32 * (i & 1)));
  }
  return 0;
}

int gpe_last_lower_flags(gpe_ctx* ctx, int64_t* n_err, int64_t* n_status) {
  if (!ctx || !n_err || !n_status) return GPE_E_INVALID;
  *n_err = ctx->lw_n_err;
  *n_status = ctx->lw_n_status;
  return 0;
}

int gpe_last_exact_host_runs(gpe_ctx* ctx, int64_t* n) {
  if (!ctx || !n) return GPE_E_INVALID;
  *n = ctx->ex_host_runs;
  return 0;
}

int gpe_last_exact_host_ms(gpe_ctx* ctx, double* ms) {
  if (!ctx || !ms) return GPE_E_INVALID;
  *ms = ctx->ex_host_ms;
  return 0;
}

#define NCCLCHK(call)                                                     \
  do {                                                                    \
    ncclResult_t r_ = (call);                                             \
    if (r_ != ncclSuccess)                                                \
      return fail(ctx, GPE_E_HIP, std::string(#call ": ") +               \
                                      rccl().error_string(r_));           \
  } while (0)

int gpe_comm_unique_id(void* id_out) {
  if (!id_out) return GPE_E_INVALID;
  RcclApi& r = rccl();
  if (!r.ok) return GPE_E_STATE;
  ncclUniqueId id;
  if (r.get_unique_id(&id) != ncclSuccess) return GPE_E_HIP;
  memcpy(id_out, &id, sizeof(id));
  return 0;
}

int gpe_comm_init(gpe_ctx* ctx, int rank, int world, const void* unique_id) {
  if (!ctx || !unique_id || world < 1 || rank < 0 || rank >= world)
    return GPE_E_INVALID;
  RcclApi& r = rccl();
  if (!r.ok) return fail(ctx, GPE_E_STATE, r.why);
  HIPCHK(hipSetDevice(ctx->device));
  if (ctx->comm) {
    NCCLCHK(r.comm_destroy(ctx->comm));
    ctx->comm = nullptr;
  }
  ncclUniqueId id;
  memcpy(&id, unique_id, sizeof(id));
  NCCLCHK(r.comm_init_rank(&ctx->comm, world, id, rank));
  ctx->comm_aborted = false;
  ctx->comm_rank = rank;
  ctx->comm_world = world;
  for (auto& e : ctx->ev_comm)
    if (!e) HIPCHK(hipEventCreate(&e));
  return 0;
}

int gpe_comm_info(const gpe_ctx* ctx, int* rank, int* world) {
  if (!ctx) return GPE_E_INVALID;
  if (rank) *rank = ctx->comm ? ctx->comm_rank : -1;
  if (world) *world = ctx->comm ? ctx->comm_world : 0;
  return 0;
}

int gpe_run_sharded_device(gpe_ctx* ctx, int mode, int64_t case_offset,
                           void* d_hi, void* d_lo, void* d_err,
                           void* d_flags) {
  if (!ctx || case_offset < 0) return GPE_E_INVALID;
  if (!ctx->comm)
    return ctx->comm_aborted
               ? fail(ctx, GPE_E_COMM, "communicator aborted (a collective timed out); "
                                       "gpe_comm_init again")
               : fail(ctx, GPE_E_STATE, "gpe_comm_init first");
  if (mode == GPE_MODE_SSE_NUMPY || mode == GPE_MODE_SSE_SEQ)
    return fail(ctx, GPE_E_INVALID,
                "order-exact sums (numpy, builtin sum) are single-device reductions");
  HIPCHK(hipSetDevice(ctx->device));
  const int64_t n = ctx->n_prog;
  const int W = ctx->comm_world;
  if (n <= 0) return 0;
  if (ensure(ctx, &ctx->d_pair, &ctx->pair_cap, (size_t)2 * n) ||
      ensure(ctx, &ctx->d_gather, &ctx->gather_cap, (size_t)W * 2 * n) ||
      ensure(ctx, &ctx->d_hi, &ctx->hi_cap, (size_t)n) ||
      ensure(ctx, &ctx->d_lo, &ctx->lo_cap, (size_t)n) ||
      ensure(ctx, &ctx->d_err, &ctx->err_cap, (size_t)n) ||
      ensure(ctx, &ctx->d_flags, &ctx->flags_cap, (size_t)n))
    return GPE_E_HIP;
  double* hi = d_hi ? (double*)d_hi : ctx->d_hi;
  double* lo = d_lo ? (double*)d_lo : ctx->d_lo;
  unsigned long long* err = d_err ? (unsigned long long*)d_err : ctx->d_err;
  uint32_t* flags = d_flags ? (uint32_t*)d_flags : ctx->d_flags;
  if (!ctx->d_ncount) HIPCHK(hipMalloc((void**)&ctx->d_ncount, 2 * sizeof(int64_t)));
  ctx->redo_global = 1;
  int rc = run_mode(ctx, mode, ctx->d_pair, ctx->d_pair + n, err, flags);
  ctx->redo_global = 0;
  if (rc) return rc;
  const unsigned blocks = (unsigned)((n + 255) / 256);
  hipLaunchKernelGGL(shard_prep, dim3(blocks), dim3(256), 0, ctx->stream, err,
                     flags, n, (uint64_t)case_offset);
  HIPCHK(hipGetLastError());
  // this rank's case count, summed over the ranks below: the MSE divisor of
  // a resident tournament after this run
  hipLaunchKernelGGL(set_i64, dim3(1), dim3(1), 0, ctx->stream, ctx->d_ncount,
                     (int64_t)ctx->n_cases);
  HIPCHK(hipGetLastError());
  RcclApi& r = rccl();
  HIPCHK(hipEventRecord(ctx->ev_comm[0], ctx->stream));
  NCCLCHK(r.group_start());
  NCCLCHK(r.all_gather(ctx->d_pair, ctx->d_gather, (size_t)2 * n, ncclFloat64,
                       ctx->comm, ctx->stream));
  NCCLCHK(r.all_reduce(err, err, (size_t)n, ncclUint64, ncclMin, ctx->comm,
                       ctx->stream));
  NCCLCHK(r.all_reduce(flags, flags, (size_t)n, ncclUint32, ncclSum, ctx->comm,
                       ctx->stream));
  NCCLCHK(r.all_reduce(ctx->d_ncount, ctx->d_ncount + 1, 1, ncclInt64, ncclSum,
                       ctx->comm, ctx->stream));
  NCCLCHK(r.group_end());
  HIPCHK(hipEventRecord(ctx->ev_comm[1], ctx->stream));
  ctx->comm_timed = true;
  hipLaunchKernelGGL(shard_finish, dim3(blocks), dim3(256), 0, ctx->stream,
                     ctx->d_gather, W, n, hi, lo, flags);
  HIPCHK(hipGetLastError());
  if (!d_hi && !d_lo && !d_err && !d_flags) keep_resident(ctx, mode, true);
  return 0;
}

int gpe_debug_shard_combine(gpe_ctx* ctx, int world, int64_t n, const double* parts,
                            const uint64_t* errs, const uint32_t* flags,
                            const int64_t* case_offsets, double* out_hi, double* out_lo,
                            uint64_t* out_err, uint32_t* out_flags) {
  if (!ctx || world < 1 || world > 1023 || n < 0 || !parts || !errs || !flags ||
      !case_offsets || !out_hi || !out_lo || !out_err || !out_flags)
    return GPE_E_INVALID;
  if (n == 0) return 0;
  HIPCHK(hipSetDevice(ctx->device));
  const size_t W = (size_t)world;
  std::vector<void*> own;
  auto alloc = [&](size_t bytes) -> void* {
    void* p = nullptr;
    if (hipMalloc(&p, bytes) != hipSuccess) return nullptr;
    own.push_back(p);
    return p;
  };
  auto release = [&]() {
    for (void* p : own) (void)hipFree(p);
  };
  double* d_gather = (double*)alloc(W * 2 * n * sizeof(double));
  unsigned long long* d_err_r = (unsigned long long*)alloc(W * n * 8);
  uint32_t* d_flags_r = (uint32_t*)alloc(W * n * 4);
  double* d_hi = (double*)alloc(n * 8);
  double* d_lo = (double*)alloc(n * 8);
  unsigned long long* d_err = (unsigned long long*)alloc(n * 8);
  uint32_t* d_flags = (uint32_t*)alloc(n * 4);
  if (own.size() != 7 || std::find(own.begin(), own.end(), nullptr) != own.end()) {
    release();
    return fail(ctx, GPE_E_HIP, "gpe_debug_shard_combine: allocation failed");
  }
  int rc = 0;
  auto step = [&]() -> int {
    HIPCHK(hipMemcpy(d_gather, parts, W * 2 * n * sizeof(double), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(d_err_r, errs, W * n * 8, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(d_flags_r, flags, W * n * 4, hipMemcpyHostToDevice));
    const unsigned blocks = (unsigned)((n + 255) / 256);
    // each rank's own preparation (gpe_run_sharded_device: shard_prep)
    for (size_t r = 0; r < W; ++r) {
      hipLaunchKernelGGL(shard_prep, dim3(blocks), dim3(256), 0, ctx->stream,
                         d_err_r + r * n, d_flags_r + r * n, n, (uint64_t)case_offsets[r]);
      HIPCHK(hipGetLastError());
    }
    // the collectives' results (RCCL all-reduce MIN / SUM), then the combine
    hipLaunchKernelGGL(emulate_rank_reduce, dim3(blocks), dim3(256), 0, ctx->stream,
                       (const unsigned long long*)d_err_r, (const uint32_t*)d_flags_r,
                       world, n, d_err, d_flags);
    HIPCHK(hipGetLastError());
    hipLaunchKernelGGL(shard_finish, dim3(blocks), dim3(256), 0, ctx->stream,
                       (const double*)d_gather, world, n, d_hi, d_lo, d_flags);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(ctx->stream));
    HIPCHK(hipMemcpy(out_hi, d_hi, n * 8, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(out_lo, d_lo, n * 8, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(out_err, d_err, n * 8, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(out_flags, d_flags, n * 4, hipMemcpyDeviceToHost));
    return 0;
  };
  rc = step();
  release();
  return rc;
}

int gpe_debug_redo_union(gpe_ctx* ctx, const uint32_t* flags, int64_t n) {
  if (!ctx || n < 0 || (n && !flags)) return GPE_E_INVALID;
  ctx->debug_redo_or.assign(flags, flags + n);
  return 0;
}

int gpe_run_sharded(gpe_ctx* ctx, int mode, int64_t case_offset, double* out_hi,
                    double* out_lo, uint64_t* out_err, uint32_t* out_flags) {
  int rc = gpe_run_sharded_device(ctx, mode, case_offset, nullptr, nullptr,
                                  nullptr, nullptr);
  if (rc) return rc;
  const size_t n = (size_t)ctx->n_prog;
  if (!n) return 0;
  if ((rc = comm_sync(ctx, "gpe_run_sharded"))) return rc;
  if (int rc_d = results_to_host(ctx, n, out_hi, out_lo, out_err, out_flags)) return rc_d;
  return 0;
}

int gpe_run_gathered(gpe_ctx* ctx, int mode, int64_t width,
                     const uint8_t* tags, double* out_hi, double* out_lo,
                     uint64_t* out_err, uint32_t* out_flags) {
  if (!ctx || width < 0) return GPE_E_INVALID;
  if (!ctx->comm)
    return ctx->comm_aborted
               ? fail(ctx, GPE_E_COMM, "communicator aborted (a collective timed out); "
                                       "gpe_comm_init again")
               : fail(ctx, GPE_E_STATE, "gpe_comm_init first");
  if (ctx->n_prog > width)
    return fail(ctx, GPE_E_INVALID, "more programs than the gather width");
  HIPCHK(hipSetDevice(ctx->device));
  const int64_t n = ctx->n_prog;
  const int W = ctx->comm_world;
  if (width == 0) return 0;
  if (ensure(ctx, &ctx->d_hi, &ctx->hi_cap, (size_t)std::max<int64_t>(n, 1)) ||
      ensure(ctx, &ctx->d_lo, &ctx->lo_cap, (size_t)std::max<int64_t>(n, 1)) ||
      ensure(ctx, &ctx->d_err, &ctx->err_cap, (size_t)std::max<int64_t>(n, 1)) ||
      ensure(ctx, &ctx->d_flags, &ctx->flags_cap, (size_t)std::max<int64_t>(n, 1)) ||
      ensure(ctx, &ctx->d_pack, &ctx->pack_cap, (size_t)4 * width) ||
      ensure(ctx, &ctx->d_gather, &ctx->gather_cap, (size_t)W * 4 * width))
    return GPE_E_HIP;
  uint8_t* d_tags = nullptr;
  if (tags && n > 0) {
    if (ensure(ctx, &ctx->d_tags, &ctx->tags_cap, (size_t)n)) return GPE_E_HIP;
    const HostPiece pc[1] = {{ctx->d_tags, tags, (size_t)n}};
    if (int rc = h2d_staged(ctx, pc, 1)) return rc;
    d_tags = ctx->d_tags;
  }
  if (n > 0) {
    int rc = run_mode(ctx, mode, ctx->d_hi, ctx->d_lo, ctx->d_err, ctx->d_flags);
    if (rc) return rc;
  }
  hipLaunchKernelGGL(pack_results, dim3((unsigned)((width + 255) / 256)), dim3(256),
                     0, ctx->stream, ctx->d_hi, ctx->d_lo, ctx->d_err,
                     ctx->d_flags, d_tags, n, width, ctx->d_pack);
  HIPCHK(hipGetLastError());
  RcclApi& r = rccl();
  HIPCHK(hipEventRecord(ctx->ev_comm[0], ctx->stream));
  NCCLCHK(r.all_gather(ctx->d_pack, ctx->d_gather, (size_t)4 * width, ncclUint64,
                       ctx->comm, ctx->stream));
  HIPCHK(hipEventRecord(ctx->ev_comm[1], ctx->stream));
  ctx->comm_timed = true;
  // into pinned staging (the tags' upload before it is stream-ordered), then
  // unpacked by host threads (a pageable destination has the runtime pin it
  // first: the stall of DESIGN 6.8)
  const size_t gbytes = (size_t)W * 4 * width * sizeof(uint64_t);
  const uint64_t* h = (const uint64_t*)pinned_buf(&ctx->h_pin_in, &ctx->h_pin_in_cap, gbytes);
  if (!h) return fail(ctx, GPE_E_HIP, "hipHostMalloc (gathered results)");
  HIPCHK(hipMemcpyAsync((void*)h, ctx->d_gather, gbytes, hipMemcpyDeviceToHost, ctx->stream));
  if (int rc = comm_sync(ctx, "gpe_run_gathered")) return rc;
  const int64_t total = (int64_t)W * width;
  const int nth = total >= 262144 ? host_threads() : 1;
  hostpool::par_run(nth, [&](int t) {
    for (int64_t o = total * t / nth, e = total * (t + 1) / nth; o < e; ++o) {
      const int64_t rk = o / width, i = o - rk * width;
      const uint64_t* g = h + (size_t)rk * 4 * width;
      if (out_hi) memcpy(&out_hi[o], &g[i], 8);
      if (out_lo) memcpy(&out_lo[o], &g[width + i], 8);
      if (out_err) out_err[o] = g[2 * width + i];
      if (out_flags) out_flags[o] = (uint32_t)g[3 * width + i];
    }
  });
  return 0;
}

int gpe_last_comm_timing(gpe_ctx* ctx, float* ms) {
  if (!ctx || !ms) return GPE_E_INVALID;
  ms[0] = ms[1] = 0.0f;
  if (ctx->comm_timed) {
    if (int rc = comm_sync(ctx, "gpe_last_comm_timing")) return rc;
    HIPCHK(hipEventElapsedTime(&ms[0], ctx->ev_comm[0], ctx->ev_comm[1]));
  }
  if (ctx->redo_timed) HIPCHK(hipEventElapsedTime(&ms[1], ctx->ev_comm[2], ctx->ev_comm[3]));
  return 0;
}

int gpe_debug_bounded_wait(double timeout_s, int64_t busy_polls, char* msg, size_t n) {
  int64_t polls = 0;
  const int rc = bounded_wait(timeout_s, [&]() {
    return (busy_polls >= 0 && polls++ >= busy_polls) ? 0 : 1;
  });
  if (msg && n)
    snprintf(msg, n, "%s",
             rc == GPE_E_COMM ? comm_timeout_msg("debug wait", 0, 1, timeout_s,
                                                 "unhandled system error").c_str()
                              : "");
  return rc;
}

int gpe_last_timing(const gpe_ctx* ctx, float* ms) {
  if (!ctx || !ms) return GPE_E_INVALID;
  ms[0] = ctx->ms[0];
  ms[1] = ctx->ms[1];
  ms[2] = ctx->ms[2];
  return 0;
}

int gpe_lexicase(gpe_ctx* ctx, const double* values, int64_t n, int64_t n_cases,
                 const uint8_t* maximise, int mode, double epsilon,
                 uint32_t* mt_state, int64_t k, int32_t* out, int64_t* failed) {
  if (!ctx || !maximise || !out || !mt_state || k < 0 || mode < 0 || mode > 2)
    return GPE_E_INVALID;
  HIPCHK(hipSetDevice(ctx->device));
  if (mt_state[kMtN] > (uint32_t)kMtN)
    return fail(ctx, GPE_E_INVALID, "lexicase: MT19937 position beyond 624");
  const double* d_val = nullptr;
  if (!values) {                    // the matrix of the last gpe_run_cases
    if (!ctx->d_case_out || ctx->n_prog <= 0)
      return fail(ctx, GPE_E_STATE, "no per-case values on the device");
    n = ctx->n_prog;
    n_cases = ctx->n_cases;
    d_val = ctx->d_case_out;
  }
  if (n <= 0 || n_cases <= 0 || n > INT32_MAX || n_cases >= (1ll << 31))
    return fail(ctx, GPE_E_INVALID, "lexicase: empty or oversized input");
  if (mode == 2 && n > 16384)
    return fail(ctx, GPE_E_INVALID,
                "automatic epsilon-lexicase on the device: at most 16384 individuals");
  const size_t lds = (size_t)((n + 31) / 32) * 4 + (size_t)n_cases * 4;
  if (lds > 48 * 1024)
    return fail(ctx, GPE_E_INVALID, "lexicase: n/32 + n_cases words exceed 48 KiB of LDS");
  // context-owned scratch (grown as needed, freed with the context)
  if ((values && ensure(ctx, &ctx->d_lex_val, &ctx->lex_val_cap, (size_t)n * n_cases)) ||
      ensure(ctx, &ctx->d_lex_max, &ctx->lex_max_cap, (size_t)n_cases) ||
      ensure(ctx, &ctx->d_sel_out, &ctx->sel_out_cap, (size_t)std::max<int64_t>(k, 1)) ||
      ensure(ctx, &ctx->d_sel_state, &ctx->sel_state_cap, (size_t)kMtN + 2) ||
      ensure(ctx, &ctx->d_lex_status, &ctx->lex_status_cap, 1) ||
      ensure(ctx, &ctx->d_lex_scratch, &ctx->lex_scratch_cap,
             (size_t)(mode == 2 ? 2 * n : 1)))
    return GPE_E_HIP;
  if (values) {
    HIPCHK(hipMemcpyAsync(ctx->d_lex_val, values, (size_t)n * n_cases * sizeof(double),
                          hipMemcpyHostToDevice, ctx->stream));
    d_val = ctx->d_lex_val;
  }
  HIPCHK(hipMemcpyAsync(ctx->d_lex_max, maximise, (size_t)n_cases, hipMemcpyHostToDevice,
                        ctx->stream));
  HIPCHK(hipMemcpyAsync(ctx->d_sel_state, mt_state, (kMtN + 1) * sizeof(uint32_t),
                        hipMemcpyHostToDevice, ctx->stream));
  HIPCHK(hipFuncSetAttribute((const void*)lexicase_mt,
                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipLaunchKernelGGL(lexicase_mt, dim3(1), dim3(kLexBlock), lds, ctx->stream, d_val,
                     n, n_cases, ctx->d_lex_max, mode, epsilon, ctx->d_sel_state, k,
                     ctx->d_sel_out, ctx->d_lex_status, ctx->d_lex_scratch);
  HIPCHK(hipGetLastError());
  int64_t st = -1;
  HIPCHK(hipMemcpyAsync(&st, ctx->d_lex_status, sizeof(int64_t), hipMemcpyDeviceToHost,
                        ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  const int64_t done = st >= 0 ? st : k;
  if (done)
    HIPCHK(hipMemcpy(out, ctx->d_sel_out, (size_t)done * sizeof(int32_t),
                     hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(mt_state, ctx->d_sel_state, (kMtN + 1) * sizeof(uint32_t),
                   hipMemcpyDeviceToHost));
  if (failed) *failed = st;
  return 0;
}

int gpe_tournament(gpe_ctx* ctx, const double* wvalues, int64_t n, int nobj,
                   double weight, int64_t k, int tournsize, uint32_t* mt_state,
                   int32_t* out) {
  if (!ctx || !mt_state || (k > 0 && !out) || k < 0 || tournsize < 1 || nobj < 1)
    return GPE_E_INVALID;
  HIPCHK(hipSetDevice(ctx->device));
  if (mt_state[kMtN] > (uint32_t)kMtN)
    return fail(ctx, GPE_E_INVALID, "tournament: MT19937 position beyond 624");
  if (!wvalues) {
    // the fitness a gpe_run / gpe_run_cases / gpe_run_device (own buffers) /
    // gpe_run_sharded_device (own buffers) left on the device, for the
    // programs and cases still loaded
    if (ctx->last_mode < 0 || ctx->last_n != ctx->n_prog || ctx->n_prog <= 0)
      return fail(ctx, GPE_E_STATE,
                  "no fitness of the loaded programs in the context's buffers "
                  "(run with the context's own outputs first)");
    n = ctx->n_prog;
    nobj = 1;
  }
  if (n <= 0 || n > INT32_MAX) return fail(ctx, GPE_E_INVALID, "tournament: no individuals");
  if (k > (int64_t)INT32_MAX / tournsize)
    return fail(ctx, GPE_E_INVALID, "tournament: k * tournsize beyond 2^31");
  if (k == 0) return 0;
  const int64_t total = k * tournsize;
  if (ensure(ctx, &ctx->d_sel_wv, &ctx->sel_wv_cap, (size_t)n * nobj) ||
      ensure(ctx, &ctx->d_sel_draws, &ctx->sel_draws_cap, (size_t)total) ||
      ensure(ctx, &ctx->d_sel_out, &ctx->sel_out_cap, (size_t)k) ||
      ensure(ctx, &ctx->d_sel_state, &ctx->sel_state_cap, (size_t)kMtN + 2))
    return GPE_E_HIP;
  uint32_t* d_status = ctx->d_sel_state + kMtN + 1;
  if (wvalues) {
    HIPCHK(hipMemcpyAsync(ctx->d_sel_wv, wvalues, (size_t)n * nobj * sizeof(double),
                          hipMemcpyHostToDevice, ctx->stream));
  } else {
    const int m = ctx->last_mode;
    const bool mse = m == GPE_MODE_MSE;
    const bool raises = mse || m == GPE_MODE_SSE_SEQ;
    HIPCHK(hipMemsetAsync(d_status, 0, sizeof(uint32_t), ctx->stream));
    hipLaunchKernelGGL(fitness_wvalues, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       ctx->stream, ctx->d_hi, ctx->d_lo, ctx->d_err, ctx->d_flags, n,
                       mse ? 1 : 0, raises ? 1 : 0,
                       ctx->last_cases_dev ? (const int64_t*)ctx->d_ncount + 1 : nullptr,
                       ctx->last_cases, weight, ctx->d_sel_wv, d_status);
    HIPCHK(hipGetLastError());
    uint32_t st = 0;
    HIPCHK(hipMemcpyAsync(&st, d_status, sizeof(uint32_t), hipMemcpyDeviceToHost,
                          ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    if (st)
      return fail(ctx, GPE_E_STATE,
                  "tournament: an individual's evaluation raises (the reference "
                  "stops before selection)");
  }
  HIPCHK(hipMemcpyAsync(ctx->d_sel_state, mt_state, (kMtN + 1) * sizeof(uint32_t),
                        hipMemcpyHostToDevice, ctx->stream));
  hipLaunchKernelGGL(tournament_draws, dim3(1), dim3(kLexBlock), 0, ctx->stream,
                     ctx->d_sel_state, n, total, ctx->d_sel_draws);
  HIPCHK(hipGetLastError());
  hipLaunchKernelGGL(tournament_pick, dim3((unsigned)((k + 255) / 256)), dim3(256), 0,
                     ctx->stream, ctx->d_sel_wv, nobj, ctx->d_sel_draws, k, tournsize,
                     ctx->d_sel_out);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(out, ctx->d_sel_out, (size_t)k * sizeof(int32_t),
                        hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipMemcpyAsync(mt_state, ctx->d_sel_state, (kMtN + 1) * sizeof(uint32_t),
                        hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  return 0;
}

int gpe_math_probe(gpe_ctx* ctx, int fn, const double* x, double* y,
                   int64_t n) {
  if (!ctx || !x || !y || n < 0 || fn < 0 || fn > 14) return GPE_E_INVALID;
  HIPCHK(hipSetDevice(ctx->device));
  double *dx = nullptr, *dy = nullptr;
  uint32_t* dcode = nullptr;
  HIPCHK(hipMalloc(&dx, std::max<int64_t>(n, 1) * sizeof(double)));
  HIPCHK(hipMalloc(&dy, std::max<int64_t>(n, 1) * sizeof(double)));
  HIPCHK(hipMemcpy(dx, x, n * sizeof(double), hipMemcpyHostToDevice));
  if (fn == 7 || fn == 8) {
    if (init_asm(ctx)) return GPE_E_HIP;
    uint32_t words[asmcore::WINDOW];
    for (auto& wd : words) wd = ctx->jump_vals32[asmcore::H_END];
    words[0] = ctx->jump_vals32[asmcore::H_LDV0];
    words[1] = ctx->jump_vals32[fn == 7 ? asmcore::H_SIN : asmcore::H_COS];
    HIPCHK(hipMalloc(&dcode, sizeof(words)));
    HIPCHK(hipMemcpy(dcode, words, sizeof(words), hipMemcpyHostToDevice));
    const int64_t per = asmcore32::K * 64;
    if (n)
      hipLaunchKernelGGL(asm_values32, dim3((unsigned)((n + per - 1) / per)),
                         dim3(64), per * sizeof(float), ctx->stream,
                         ctx->d_cst32, dcode, dx, dy, n, fn == 8, nullptr);
  } else if (fn == 13 || fn == 14) {
    if (init_asm(ctx)) return GPE_E_HIP;
    uint32_t words[asmcore::WINDOW];
    for (auto& wd : words) wd = ctx->jump_vals_exact[asmcore::H_END];
    words[0] = ctx->jump_vals_exact[asmcore::H_LDV0];
    words[1] = ctx->jump_vals_exact[fn == 13 ? asmcore::H_SIN : asmcore::H_COS];
    HIPCHK(hipMalloc(&dcode, sizeof(words)));
    HIPCHK(hipMemcpy(dcode, words, sizeof(words), hipMemcpyHostToDevice));
    const int64_t per = asmcore_exact::K * 64;
    if (n)
      hipLaunchKernelGGL(asm_values_exact, dim3((unsigned)((n + per - 1) / per)),
                         dim3(64), asmcore_exact::GLIBC_LDS_BYTES + per * sizeof(double),
                         ctx->stream, ctx->d_cst_exact, dcode, dx, dy, n, fn == 14,
                         nullptr);
  } else if (fn == 5 || fn == 6) {
    if (init_asm(ctx)) return GPE_E_HIP;
    uint32_t words[asmcore::WINDOW];
    for (auto& wd : words) wd = ctx->jump_vals[asmcore::H_END];
    words[0] = ctx->jump_vals[asmcore::H_LDV0];
    words[1] = ctx->jump_vals[fn == 5 ? asmcore::H_SIN : asmcore::H_COS];
    HIPCHK(hipMalloc(&dcode, sizeof(words)));
    HIPCHK(hipMemcpy(dcode, words, sizeof(words), hipMemcpyHostToDevice));
    const int64_t per = asmcore::K * 64;
    if (n)
      hipLaunchKernelGGL(asm_values, dim3((unsigned)((n + per - 1) / per)),
                         dim3(64), kTrigLdsBytes + per * sizeof(double),
                         ctx->stream, ctx->d_cst, dcode, dx, dy, n, fn == 6, nullptr);
  } else if (n) {
    hipLaunchKernelGGL(math_probe, dim3((unsigned)((n + 255) / 256)),
                       dim3(256), 0, ctx->stream, fn, dx, dy, n);
  }
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(ctx->stream));
  if (dcode) HIPCHK(hipFree(dcode));
  HIPCHK(hipMemcpy(y, dy, n * sizeof(double), hipMemcpyDeviceToHost));
  HIPCHK(hipFree(dx));
  HIPCHK(hipFree(dy));
  return 0;
}

int gpe_host_np_sum(const double* x, int64_t n_rows, int64_t n_cols,
                    double* out) {
  if ((!x && n_rows * n_cols) || !out || n_rows < 0 || n_cols <= 0)
    return GPE_E_INVALID;
  const NpPlan p = np_plan(n_cols);
  if (p.depth > kNpStack) return GPE_E_INVALID;
  std::vector<double> leaf(p.off.size());
  double st[kNpStack];
  for (int64_t r = 0; r < n_rows; ++r) {
    const double* row = x + r * n_cols;
    for (size_t i = 0; i < p.off.size(); ++i) leaf[i] = np_leaf(row + p.off[i], p.len[i]);
    out[r] = np_combine(p.post.data(), (int)p.post.size(), leaf.data(), st);
  }
  return 0;
}

int gpe_host_math(int fn, const double* x, double* y, int64_t n) {
  if (!x || !y || n < 0 || fn < 0 || fn > 8) return GPE_E_INVALID;
  if (fn >= 7) {                          // glibc_trig_k<2>: two at a time
    for (int64_t i = 0; i < n; i += 2) {
      double v[2] = {x[i], i + 1 < n ? x[i + 1] : 0.0};
      glibc_trig_k<2>(v, fn == 8, asmcore::kGlibcSincostab, asmcore::kGlibcToverp);
      y[i] = v[0];
      if (i + 1 < n) y[i + 1] = v[1];
    }
    return 0;
  }
  if (fn >= 5) {                          // glibc_sin / glibc_cos
    for (int64_t i = 0; i < n; ++i) y[i] = glibc_trig(x[i], fn == 6);
    return 0;
  }
  if (fn >= 3) {                          // fp32 mode's gp_trig32
    for (int64_t i = 0; i < n; ++i) y[i] = gp_trig32((float)x[i], fn == 4);
    return 0;
  }
  for (int64_t i = 0; i < n; ++i) {
    double sn, cs;
    gp_sincos(x[i], sn, cs);
    y[i] = fn == 0 ? sn : fn == 1 ? cs : x[i] * x[i];
  }
  return 0;
}

int gpe_debug_translate(const uint32_t* code, int64_t n_words,
                        const int64_t* off, int64_t n_prog,
                        const int32_t* depth, int nv, const uint32_t* table,
                        int n_table, uint32_t* out, int64_t out_cap,
                        int64_t* starts, int64_t* n_out) {
  if (!code || !off || !depth || !table || !out || !starts || !n_out ||
      (n_table != asmcore::H_COUNT && n_table != asmcore_deep::H_COUNT))
    return GPE_E_INVALID;
  // the table's size names the core: D = 5 (programs it holds) or deep
  const bool deep_core = n_table == asmcore_deep::H_COUNT;
  std::vector<uint32_t> tab(table, table + n_table), acode;
  for (int64_t i = 0; i < n_prog; ++i) {
    bool ok = false;
    if (off[i] < 0 || off[i + 1] > n_words || off[i + 1] <= off[i])
      return GPE_E_INVALID;
    if (!validate_program(code + off[i], off[i + 1] - off[i], GPE_MACHINE_F,
                          nv, depth[i], &ok).empty())
      return GPE_E_INVALID;
    starts[i] = -1;
    if (!ok || (!deep_core && depth[i] > asmcore::D)) continue;
    starts[i] = (int64_t)acode.size();
    translate_program(code + off[i], tab, acode, false, deep_core ? kIdsDeep : kIds);
  }
  if ((int64_t)acode.size() > out_cap) return GPE_E_INVALID;
  std::copy(acode.begin(), acode.end(), out);
  *n_out = (int64_t)acode.size();
  return 0;
}

int gpe_last_geometry(const gpe_ctx* ctx, int64_t* o) {
  if (!ctx || !o) return GPE_E_INVALID;
  o[0] = ctx->fasm.programs + ctx->dasm.programs;
  o[1] = ctx->fast.programs;
  o[2] = ctx->deep.programs;
  o[3] = ctx->redo_programs;
  // the D = 5 asm launch as it ran: the exact core's (every fp64 MSE run by
  // default) or the table core's
  const Launch& A = ctx->last_exact_all ? ctx->redo_xasm : ctx->fasm;
  o[4] = ctx->fasm.programs ? A.P : ctx->fast.P;
  o[5] = ctx->fasm.programs ? A.groups : ctx->fast.groups;
  o[6] = ctx->redo_tiles;
  o[7] = ctx->fasm.programs ? A.wpb : ctx->fast.wpb;
  return 0;
}

int gpe_last_geometry_ex(const gpe_ctx* ctx, int64_t* o, int n) {
  if (!ctx || !o || n < 0) return GPE_E_INVALID;
  int64_t g[GPE_GEOMETRY_FIELDS];
  gpe_last_geometry(ctx, g);
  const Launch& D = ctx->last_exact_all ? ctx->redo_xasm_deep : ctx->dasm;
  g[8] = ctx->dasm.programs;
  g[9] = D.P;
  g[10] = D.groups;
  g[11] = D.wpb;
  g[12] = ctx->redo_exact_cpp;
  g[13] = ctx->tasm.programs;        // the typed core (HITS_BOOL)
  g[14] = ctx->tasm.P;
  g[15] = ctx->tasm.groups;
  g[16] = ctx->planned_mode == GPE_MODE_HITS_BOOL ? ctx->n_kc : 0;   // constants: no core run
  std::copy(g, g + std::min(n, GPE_GEOMETRY_FIELDS), o);
  return 0;
}

}  // extern "C"
