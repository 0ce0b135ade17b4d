// Part of gpeval.hip's single translation unit (included there once, in
// order, inside the library's anonymous namespace for device code): the multi-GPU layer — the device combine
// kernels of case sharding and RCCL opened with dlopen.
#pragma once
namespace {

// ------------------------------------------------- multi-GPU (RCCL) ----
// Case sharding (gpe_run_sharded*): every rank evaluates all programs on its
// slice of the cases; the per-program partials are combined on the device:
// the (hi, lo) double-doubles are all-gathered and summed in rank order
// (deterministic, the order distributed.py's host fallback uses), the
// first-error code is all-reduced with MIN after adding the rank's case
// offset, and the three flag bits are OR-ed through one SUM of 10-bit fields.
__global__ void shard_prep(unsigned long long* err, uint32_t* flags, int64_t n,
                           uint64_t case_offset) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const unsigned long long e = err[i];
  if (e != ~0ull) err[i] = e + (case_offset << 2);
  const uint32_t f = flags[i];
  flags[i] = (f & 1u) | ((f & 2u) << 9) | ((f & 4u) << 18);
}

__global__ void shard_finish(const double* gather, int world, int64_t n,
                             double* hi, double* lo, uint32_t* flags) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double h = 0.0, l = 0.0;
  for (int r = 0; r < world; ++r) {
    const double* g = gather + (size_t)r * 2 * n;
    dd_add(h, l, g[i], g[n + i]);
  }
  hi[i] = h;
  lo[i] = l;
  const uint32_t f = flags[i];
  flags[i] = ((f & 0x3ffu) ? 1u : 0u) | (((f >> 10) & 0x3ffu) ? 2u : 0u) |
             (((f >> 20) & 0x3ffu) ? 4u : 0u);
}

// gpe_debug_shard_combine: what the all-reduces of gpe_run_sharded_device
// leave in err/flags (MIN over the ranks' prepared words, SUM of the packed
// flag counters), computed on one device from the W ranks' arrays
__global__ void emulate_rank_reduce(const unsigned long long* err_r,
                                    const uint32_t* flags_r, int world, int64_t n,
                                    unsigned long long* err, uint32_t* flags) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  unsigned long long e = ~0ull;
  uint32_t f = 0;
  for (int r = 0; r < world; ++r) {
    e = min(e, err_r[(size_t)r * n + i]);
    f += flags_r[(size_t)r * n + i];
  }
  err[i] = e;
  flags[i] = f;
}

// Population sharding (gpe_run_gathered): this rank's results packed as
// 4 words per slot, [hi | lo | err | flags | tag << 8] planes of `width`
// slots (tags: the caller's per-program byte, e.g. flattener verdicts).
__global__ void pack_results(const double* hi, const double* lo,
                             const unsigned long long* err,
                             const uint32_t* flags, const uint8_t* tags,
                             int64_t n, int64_t width, uint64_t* out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= width) return;
  uint64_t h = 0, l = 0, e = ~0ull, f = 0;
  if (i < n) {
    memcpy(&h, &hi[i], 8);
    memcpy(&l, &lo[i], 8);
    e = err[i];
    f = flags[i] | (tags ? (uint32_t)tags[i] << 8 : 0u);
  }
  out[i] = h;
  out[width + i] = l;
  out[2 * width + i] = e;
  out[3 * width + i] = f;
}

// RCCL entry points, resolved at first use (libgpeval.so does not link
// RCCL: a process that never shards needs no librccl).  Inside a torch
// process this finds the librccl.so.1 torch already loaded.
struct RcclApi {
  bool tried = false, ok = false;
  std::string why;
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRank) comm_init_rank = nullptr;
  decltype(&ncclCommDestroy) comm_destroy = nullptr;
  decltype(&ncclAllReduce) all_reduce = nullptr;
  decltype(&ncclAllGather) all_gather = nullptr;
  decltype(&ncclGroupStart) group_start = nullptr;
  decltype(&ncclGroupEnd) group_end = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
  decltype(&ncclCommAbort) comm_abort = nullptr;
  decltype(&ncclCommGetAsyncError) async_error = nullptr;
};

RcclApi& rccl() {
  static RcclApi api;
  if (api.tried) return api;
  api.tried = true;
  void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
  if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
  if (!h) {
    const char* e = dlerror();
    api.why = std::string("cannot open librccl.so.1: ") + (e ? e : "?");
    return api;
  }
  auto sym = [&](const char* name) -> void* {
    void* p = dlsym(h, name);
    if (!p && api.why.empty()) api.why = std::string("librccl: no symbol ") + name;
    return p;
  };
  api.get_unique_id = (decltype(api.get_unique_id))sym("ncclGetUniqueId");
  api.comm_init_rank = (decltype(api.comm_init_rank))sym("ncclCommInitRank");
  api.comm_destroy = (decltype(api.comm_destroy))sym("ncclCommDestroy");
  api.all_reduce = (decltype(api.all_reduce))sym("ncclAllReduce");
  api.all_gather = (decltype(api.all_gather))sym("ncclAllGather");
  api.group_start = (decltype(api.group_start))sym("ncclGroupStart");
  api.group_end = (decltype(api.group_end))sym("ncclGroupEnd");
  api.error_string = (decltype(api.error_string))sym("ncclGetErrorString");
  api.comm_abort = (decltype(api.comm_abort))sym("ncclCommAbort");
  api.async_error = (decltype(api.async_error))sym("ncclCommGetAsyncError");
  api.ok = api.why.empty();
  return api;
}

// sin/cos of every variable, evaluated once per run (gpe_set_trig_leaves):
// the flattener lowers sin(ARGv)/cos(ARGv) leaves to reads of these columns,
// computed with glibc_trig: the reference's own values, which an inline
// table sin/cos matches except where glibc misrounds.
// (fp32 mode: the fp32 sin/cos of the float argument, exactly what an
// inline sin/cos node computes there; the staged float cast is exact)
__global__ void leaf_trig(double* X, int nv, int64_t n, int f32) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n * nv) return;
  const int v = (int)(i / n);
  const int64_t c = i - (int64_t)v * n;
  const double x = X[(int64_t)v * n + c];
  // fp64: glibc 2.35's own algorithm, the reference's math.sin/cos bit for
  // bit (a leaf value is read by every program; a redo of a program cannot
  // recompute it)
  X[(int64_t)(nv + v) * n + c] = f32 ? (double)gp_trig32((float)x, false) : glibc_trig(x, false);
  X[(int64_t)(2 * nv + v) * n + c] = f32 ? (double)gp_trig32((float)x, true) : glibc_trig(x, true);
}

}  // namespace
