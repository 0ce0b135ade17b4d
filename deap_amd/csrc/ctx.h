// Part of gpeval.hip's single translation unit (included there once, in
// order): the host-side state — a launch's plan (Launch), numpy.sum's plan, the
// chunked lowering's staging, and the context (gpe_ctx) behind the C ABI.
#pragma once

// ====================================================================== host
struct Launch {
  std::vector<int32_t> slot_prog;   // host copy
  int32_t* d_slot_prog = nullptr;
  int64_t n_slots = 0;
  int P = 1;
  int sdepth = 1;                   // deepest program's stack slots (>= 1)
  int wpb = kWaves;                 // waves per block
  int64_t n_tiles = 0;
  int groups = 0;
  int tiles_per_group = 0;
  int64_t waves = 0;
  double* d_part = nullptr;
  size_t part_cap = 0;
  size_t slot_cap = 0;
  int64_t programs = 0;
  int K = 0;                        // asm launches: the core's cases per lane
  bool dbuf = false;                // asm launches: two tile buffers (asm_dbuf)
  char* h_pin = nullptr;            // pinned staging of the slot upload
  size_t h_pin_cap = 0;
};


// ------------------------------------------------------------ numpy.sum --
// numpy 2.2's float64 add.reduce over a contiguous row, restated exactly
// (the reduction examples/gp/symbreg_numpy.py:66 calls): the reduce loop is
// fed buffer chunks of 8192 elements, acc = 0.0; acc += pw(chunk) for each,
// where pw(n < 8) adds left to right from -0.0, pw(n <= 128) keeps 8
// strided accumulators r[j] (+= x[i + j]), combines them as
// ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7)) and then adds the n % 8
// tail in order, and pw(n > 128) = pw(n2) + pw(n - n2) with n2 = n / 2
// rounded down to a multiple of 8.  The recursion is unrolled on the host
// into leaves (offset, length) and a postfix program over them:
// >= 0 push leaf sum, kNpAdd pop b, a and push a + b, kNpZero push 0.0.
constexpr int32_t kNpAdd = -1, kNpZero = -2;
constexpr int64_t kNpChunk = 8192, kNpBlock = 128;
constexpr int kNpStack = 64;

HD double np_leaf(const double* x, int64_t n) {
  if (n < 8) {
    double res = -0.0;
    for (int64_t i = 0; i < n; ++i) res = res + x[i];
    return res;
  }
  double r[8];
  for (int j = 0; j < 8; ++j) r[j] = x[j];
  int64_t i = 8;
  for (; i < n - (n % 8); i += 8)
    for (int j = 0; j < 8; ++j) r[j] = r[j] + x[i + j];
  double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  for (; i < n; ++i) res = res + x[i];
  return res;
}

// Python's builtin sum over a row (examples/gp/adf_symbreg.py:124,
// sum(map(...)): 0 + x0 + x1 + ... left to right), one thread per row.
__global__ void __launch_bounds__(256)
seq_sum_rows(const double* __restrict__ rows, int64_t n_cols, int64_t n_rows,
             double* __restrict__ out_hi, double* __restrict__ out_lo) {
  const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (r >= n_rows) return;
  const double* x = rows + r * n_cols;
  double acc = 0.0;
  for (int64_t i = 0; i < n_cols; ++i) acc = acc + x[i];
  out_hi[r] = acc;
  out_lo[r] = 0.0;
}

struct NpPlan {
  std::vector<int64_t> off;
  std::vector<int32_t> len;
  std::vector<int32_t> post;
  int depth = 0;
};

inline void np_plan_rec(int64_t lo, int64_t n, NpPlan& p) {
  if (n <= kNpBlock) {
    p.post.push_back((int32_t)p.off.size());
    p.off.push_back(lo);
    p.len.push_back((int32_t)n);
    return;
  }
  int64_t n2 = n / 2;
  n2 -= n2 % 8;
  np_plan_rec(lo, n2, p);
  np_plan_rec(lo + n2, n - n2, p);
  p.post.push_back(kNpAdd);
}

inline NpPlan np_plan(int64_t n) {
  NpPlan p;
  p.post.push_back(kNpZero);
  for (int64_t c = 0; c < n; c += kNpChunk) {
    np_plan_rec(c, std::min(kNpChunk, n - c), p);
    p.post.push_back(kNpAdd);
  }
  int sp = 0;
  for (int32_t w : p.post) {
    sp += w == kNpAdd ? -1 : 1;
    p.depth = std::max(p.depth, sp);
  }
  return p;
}

HD double np_combine(const int32_t* post, int n_post, const double* leaf,
                     double* st) {
  int sp = 0;
  for (int k = 0; k < n_post; ++k) {
    const int32_t w = post[k];
    if (w >= 0) {
      st[sp++] = leaf[w];
    } else if (w == kNpZero) {
      st[sp++] = 0.0;
    } else {
      --sp;
      st[sp - 1] = st[sp - 1] + st[sp];
    }
  }
  return st[0];
}

// One wave per program: lanes sum the leaves of the program's per-case row,
// then lane 0 runs the combine program (stack in LDS).
__global__ void __launch_bounds__(64)
np_sum_rows(const double* __restrict__ rows, int64_t n_cols,
            const int64_t* __restrict__ off, const int32_t* __restrict__ len,
            int n_leaves, const int32_t* __restrict__ post, int n_post,
            double* __restrict__ leaf, double* __restrict__ out_hi,
            double* __restrict__ out_lo) {
  __shared__ double st[kNpStack];
  const int64_t r = blockIdx.x;
  const double* x = rows + r * n_cols;
  double* lf = leaf + r * n_leaves;
  for (int i = threadIdx.x; i < n_leaves; i += 64) lf[i] = np_leaf(x + off[i], len[i]);
  __syncthreads();
  if (threadIdx.x == 0) {
    out_hi[r] = np_combine(post, n_post, lf, st);
    out_lo[r] = 0.0;
  }
}

// One chunk of a device lowering (gpe_lower_add): its inputs and scratch
// on the device and its own pinned staging on the host, kept across calls.
// The chunks of one lowering run on the stream one after another while the
// caller reads the next chunk's trees.
struct LowerChunk {
  uint8_t* codes = nullptr;
  size_t codes_cap = 0;
  int64_t* node_off = nullptr;
  size_t node_off_cap = 0;
  int64_t* eph_off = nullptr;
  size_t eph_off_cap = 0;
  lowering::Val* evals = nullptr;
  size_t evals_cap = 0;
  uint16_t* l16 = nullptr;         // per tree: length, then ephemeral count
  size_t l16_cap = 0;
  lowering::PRec* rec = nullptr;
  size_t rec_cap = 0;
  int32_t* stk = nullptr;
  size_t stk_cap = 0;
  lowering::Val* cv = nullptr;
  size_t cv_cap = 0;
  double* ib = nullptr;            // int bounds of the records (F machine)
  size_t ib_cap = 0;
  uint32_t* words = nullptr;
  size_t words_cap = 0;
  int64_t* wrow = nullptr;         // interleaved scratch: per-wave row and
  size_t wrow_cap = 0;             // word-row bases (lower_trees<true>)
  int64_t* wword = nullptr;
  size_t wword_cap = 0;
  char* h_pin = nullptr;
  size_t h_pin_cap = 0;
  std::vector<int64_t> wrow_h, wword_h;
  std::vector<uint16_t> l16_h;
  int64_t start = 0, n = 0;
  bool il = false;
  hipEvent_t ev = nullptr;         // its word counts and metadata on the host
  char* scan_tmp = nullptr;        // its offset scans' temporary storage
  size_t scan_tmp_cap = 0;
};

struct gpe_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ev[3] = {nullptr, nullptr, nullptr};
  hipEvent_t ev_redo[2] = {nullptr, nullptr};   // around the redo passes
  hipEvent_t ev_lw = nullptr;      // gpe_lower_begin: the lowering streams start behind the
                                   // context stream's work
  // the chunks of a device lowering alternate between these two streams:
  // one launch of lower_trees has a ~0.4 ms floor (one wave lowering its 64
  // trees), so a chunk's tail overlaps the next chunk's start
  hipStream_t lw_stream[2] = {nullptr, nullptr};
  // around the last sharded / gathered run's collectives ([0], [1]) and the
  // case-sharded redo-flag all-reduce ([2], [3]): gpe_last_comm_timing
  hipEvent_t ev_comm[4] = {nullptr, nullptr, nullptr, nullptr};
  bool comm_timed = false, redo_timed = false;
  bool comm_aborted = false;        // a collective timed out: the communicator is gone
  std::string err;
  // cases
  int machine = -1;
  void* d_X = nullptr;
  void* d_terms = nullptr;
  int nv = 0, nt = 0;               // nv: columns the kernels see
  int nv_user = 0;                  // variables given to set_cases
  int trig_leaves = 0;              // columns [nv_user, 3 nv_user):
                                    // sin(x_v), cos(x_v) per run
  int64_t n_cases = 0, n_units = 0;
  // programs (flattener format)
  uint32_t* d_code = nullptr;
  size_t code_cap = 0;
  int64_t* d_off = nullptr;
  size_t off_cap = 0;
  int64_t n_prog = 0;
  std::vector<int32_t> cost;         // planner weight: words + trig_w * sin/cos + div_w * protectedDiv (clamped)
  std::vector<int32_t> depth;
  std::vector<uint8_t> asm_ok;       // asm core: 0 none, 1 D = 5, 2 deep
  // asm fast path
  bool asm_ready = false;
  // fp32 core (gen_asm32.py): handler table, constants, and the precision
  // the current threaded code was translated for
  std::vector<uint32_t> asm32_table;
  float* d_cst32 = nullptr;
  int acode_prec = -1;
  std::vector<uint32_t> asm_table;   // handler id -> byte offset
  std::vector<uint32_t> asm_deep_table;    // ... of the deep fp64 core
  std::vector<uint32_t> asm_exact_table;   // ... of the exact core
  double* d_cst_exact = nullptr;           // its LDS image (glibc tables)
  uint32_t* d_acode_x = nullptr;           // redo programs for the exact core
  size_t acode_x_cap = 0;
  uint32_t* d_astart_x = nullptr;
  size_t astart_x_cap = 0;
  uint32_t* d_redo2 = nullptr;             // ... it leaves to the C++ pass
  size_t redo2_cap = 0;
  uint32_t* d_redo2_count = nullptr;
  std::vector<uint32_t> asm32_deep_table;  // ... of the deep fp32 core
  // The program words each kernel's copy of a core jumps through: the low
  // half of the handler's absolute address (offset + that kernel's .Lbase,
  // probed once; gen_asm.py dispatch_head)
  std::vector<uint32_t> jump_asm, jump_asm_deep, jump_asm_exact, jump_asm32,
      jump_asm32_deep, jump_vals, jump_vals_exact, jump_vals32;
  // the typed core (HITS_BOOL): its handler table and jump words; per
  // program whether it runs there; its threaded code (translated on the
  // first HITS_BOOL run after a load)
  std::vector<uint32_t> asm_typed_table, jump_asm_typed;
  std::vector<uint32_t> asm_exact_deep_table, jump_asm_exact_deep;
  uint32_t* d_jump_asm_exact_deep = nullptr;
  std::vector<uint8_t> typed_ok;
  bool typed_valid = false;
  int use_typed = 1;                 // GPE_TYPED_ASM=0 disables (A/B testing)
  uint32_t* d_acode_t = nullptr;
  size_t acode_t_cap = 0;
  // device translation (translate_device): per-program lengths and classes,
  // and each core's jump words on the device
  uint32_t* d_xl_len = nullptr;
  size_t xl_len_cap = 0;
  uint8_t* d_xl_cls = nullptr;
  size_t xl_cls_cap = 0;
  // pinned host staging for the small device-to-host reads of every
  // generation (lowering metadata, translation lengths, typed routing):
  // pageable destinations measured up to 20 ms per read on the GPU box
  char* h_pin = nullptr;
  size_t h_pin_cap = 0;
  char* h_pin_in = nullptr;          // host→device staging of gpe_lower_programs
  size_t h_pin_in_cap = 0;
  char* h_pin_redo = nullptr;        // the redo bookkeeping's one D2H (count,
  size_t h_pin_redo_cap = 0;         // programs, compacted list head)
  uint32_t* d_redo_nsel = nullptr;   // flagged programs (DeviceSelect count)
  uint32_t *d_jump_asm = nullptr, *d_jump_asm_deep = nullptr, *d_jump_asm_exact = nullptr,
           *d_jump_asm32 = nullptr, *d_jump_asm32_deep = nullptr, *d_jump_asm_typed = nullptr;
  uint32_t* d_astart_t = nullptr;
  size_t astart_t_cap = 0;
  double* d_cst = nullptr;
  uint32_t* d_acode = nullptr;
  size_t acode_cap = 0;
  uint32_t* d_astart = nullptr;
  size_t astart_cap = 0;
  uint32_t* d_redo = nullptr;
  size_t redo_cap = 0;
  uint32_t* d_redo_count = nullptr;
  uint64_t* d_redo_list = nullptr;   // (program, tile) pairs of the asm core
  uint32_t redo_list_cap = 0;
  double* d_pair_part = nullptr;
  size_t pair_part_cap = 0;
  uint64_t* d_pair_sorted = nullptr;  // redo_pairs: the sorted pair list,
  size_t pair_sorted_cap = 0;         // each program's first pair,
  int64_t* d_pair_off = nullptr;      // their count, the sort's scratch
  size_t pair_off_cap = 0;
  uint32_t* d_pair_nruns = nullptr;
  size_t pair_nruns_cap = 0;
  char* d_sort_tmp = nullptr;
  size_t sort_tmp_cap = 0;
  int use_asm = 1;                   // GPE_ASM=0 disables (A/B testing)
  int asm_pmax = 8;            // programs per wave (asm kernel), LDS permitting
  int typed_pmax = 64;         // ... of the typed core (GPE_TYPED_PMAX, <= 64: a lane each)
  int typed_waves = 8;         // waves per typed-core block (GPE_TYPED_WAVES)
  int64_t target_blocks = 8192;  // planner's grid target
  // ... of the asm cores' tile groups: more, smaller blocks shorten the
  // grid's tail (C4: 48 tile groups, 2% faster than 8)
  int64_t asm_target_blocks = 65536;
  int64_t xasm_target_blocks = 65536;  // ... of the exact core's redo launch
  // ... of the typed core (C5 at pop 1M: 12 tile groups at 32768 against 18
  // at 65536, kernel 3.75 -> 3.58 ms; 8 and 36 groups slower,
  // scripts/r05_typed_groups.sh)
  int64_t typed_target_blocks = 32768;
  int64_t min_group_tiles = 0;         // asm launches: tiles per group, at least (0: off)
  // a program's cost: its code words + trig_w per sin/cos node + div_w per
  // protectedDiv node (round 6 on the exact core, same box, ms per C4 step:
  // trig_w alone 0 / 4 / 8 / 14 -> 692.8 / 663.7 / 660.1 / 663.2; with div_w
  // (8, 0 / 2 / 4 / 8) -> 652.4 / 648.3 / 649.5 / 657.4; (10, 3) / (12, 4) /
  // (14, 5) / (16, 6) -> 647.8 / 647.9 / 646.7 / 647.1; scripts/r06_gpu8.sh,
  // r06_gpu12.sh .. r06_gpu14.sh)
  int trig_w = 14;
  int div_w = 5;
  // GPE_DEAL_MIX: odd waves run their programs in reverse deal order, so
  // neighbouring waves (and a CU's blocks) work on programs of different
  // cost bands at once (per-wave totals unchanged)
  int deal_mix = 0;
  int asm_waves = 8;           // waves per f_eval_asm block (share a tile)
  int asm_lds_kb = 80;         // LDS per f_eval_asm block (2 blocks per CU)
  int asm_dbuf = 1;            // two tile buffers, LDS-DMA (GPE_ASM_DBUF)
  int lw_interleave = 1;       // interleaved lowering scratch (GPE_LOWER_IL)
  int neg_fold = 1;            // lowering's NEG peephole (GPE_NEG_PEEPHOLE=0: off)
  int exact_all = 1;           // GPE_EXACT_ALL: the exact cores (0: table cores + redo)
  // gpe_debug_redo_union: redo flags "another rank" raised, ORed in where a
  // case-sharded run all-reduces them (test infrastructure)
  std::vector<uint32_t> debug_redo_or;
  int asm_deep_waves = 4;      // ... of the deep cores (fewer waves per SIMD)
  int f_waves = 8;             // C++ F kernels: 8 where LDS allows, else 4
  int b_lanes = 1;             // lane-packed B kernel for tiny case sets
  int diag = 0;                // GPE_DIAG: 1 skip epilogue, 2 stage once
  // sin/cos arguments at or past 2^(redo_exp) send the fp64 asm core's
  // (program, tile) to the redo pass (the reference's libm bit for bit);
  // GPE_REDO_EXP, default and maximum 40 (the core's own range)
  uint32_t redo_hi = (uint32_t)asmcore::LIM_HI;
  // ... of the deep core (programs needing 6..12 operand-stack slots: large
  // trees, where a last-bit sin/cos difference upstream is most often
  // amplified): 2^20 (GPE_REDO_EXP_DEEP); tests/golden/c4_deep_core.json.gz
  // has trees whose largest argument is 2^21 .. 2^37 and whose fitness the
  // table sin/cos moves by up to 7e-12 relative
  uint32_t redo_hi_deep = (uint32_t)(0x3ff + 20) << 20;
  // launch plans, rebuilt per (mode, subset)
  Launch fast, deep, fasm, dasm, tasm, redo_fast, redo_deep, redo_xasm, redo_xasm_deep;
  bool last_exact_all = false;         // the last run put its asm programs on the exact cores
  // host scratch reused across calls (per-call fresh vectors of a million
  // entries page-faulted on every generation: 20+ ms on the GPU box's host)
  std::vector<int32_t> pl_fa, pl_da, pl_ta, pl_fc, pl_dc, pl_order;
  // HITS_BOOL: programs that are one folded constant (LDC c; END — 43 % of
  // spambase.py's genHalfAndHalf(1, 2) population: not_/and_/or_ of bool
  // terminals).  Their hit count is the number of cases whose label has
  // bool(c)'s truth, label_true or n_cases - label_true: no core run.
  // pl_kc[i] = 2 * program + bool(c); label_true: labels != 0 (nan counts)
  std::vector<uint32_t> pl_kc;
  uint32_t* d_kc = nullptr;
  size_t kc_cap = 0;
  int64_t n_kc = 0;
  int64_t label_true = 0;
  std::vector<int64_t> pl_start;

  int planned_mode = -1;
  // outputs (device)
  double* d_hi = nullptr;
  double* d_lo = nullptr;
  unsigned long long* d_err = nullptr;
  uint32_t* d_flags = nullptr;
  size_t hi_cap = 0, lo_cap = 0, err_cap = 0, flags_cap = 0;
  double* d_case_out = nullptr;      // per-case output of gpe_run_cases
  size_t case_cap = 0;
  int prec = GPE_PREC_F64;           // F machine arithmetic (gpe_set_precision)
  // numpy.sum plan for n_cases (GPE_MODE_SSE_NUMPY), built on first use
  int64_t np_n = 0;
  int np_leaves = 0, np_post = 0;
  int64_t* d_np_off = nullptr;
  int32_t* d_np_len = nullptr;
  int32_t* d_np_post = nullptr;
  double* d_np_leaf = nullptr;
  size_t np_leaf_cap = 0;
  int case_on = 0;
  float ms[3] = {0, 0, 0};
  int64_t redo_programs = 0;
  int64_t redo_tiles = 0;
  int64_t redo_exact_cpp = 0;   // ... of them the exact core left to C++
  // device lowering (gpe_set_lowering / gpe_lower_programs)
  int lw_machine = -1, lw_nv = 0;
  std::vector<uint8_t> lw_leaf;
  lowering::Entry* d_lw_entries = nullptr;
  uint8_t* d_lw_leaf = nullptr;
  int lw_n_leaf = 0;
  std::vector<LowerChunk> lw_ch;     // the chunks of device lowering
  int lw_k = 0;                      // chunks added to the open lowering
  int64_t lw_total_n = 0, lw_added = 0, lw_nodes = 0;
  bool lw_open = false;              // gpe_lower_begin .. gpe_lower_end
  // gpe_lower_begin_into: the caller's per-tree outputs, filled chunk by
  // chunk as the chunks' metadata arrives (lw_dec: chunks decoded)
  int32_t* lw_out_depth = nullptr;
  uint8_t* lw_out_err = nullptr;
  uint8_t* lw_out_status = nullptr;
  int lw_dec = 0;
  bool lw_too_deep = false;
  // the last lowering's trees with a nonzero error code / status
  // (gpe_last_lower_flags: the caller skips its scans when both are 0)
  int64_t lw_n_err = 0, lw_n_status = 0;
  uint32_t* lw_hm = nullptr;         // pinned: word counts [n], metadata [n]
  size_t lw_hm_cap = 0;
  uint32_t* d_lw_nw = nullptr;
  size_t lw_nw_cap = 0;
  uint32_t* d_lw_meta = nullptr;
  size_t lw_meta_cap = 0;
  // the last run's device outputs (gpe_tournament without host values):
  // only the context's own buffers, and only until the programs or cases
  // change (last_mode < 0: nothing resident)
  int last_mode = -1;
  int64_t last_n = 0;
  double last_cases = 0.0;            // the MSE divisor ...
  bool last_cases_dev = false;        // ... or d_ncount (case-sharded runs)
  int64_t* d_ncount = nullptr;        // [0] local case count, [1] all-reduced
  // scratch of the selection kernels and the redo pass (grown, never freed
  // per call)
  double* d_sel_wv = nullptr;
  size_t sel_wv_cap = 0;
  int32_t* d_sel_draws = nullptr;
  size_t sel_draws_cap = 0;
  int32_t* d_sel_out = nullptr;
  size_t sel_out_cap = 0;
  uint32_t* d_sel_state = nullptr;     // MT19937 state + position, then status
  size_t sel_state_cap = 0;
  double* d_lex_val = nullptr;
  size_t lex_val_cap = 0;
  uint8_t* d_lex_max = nullptr;
  size_t lex_max_cap = 0;
  int64_t* d_lex_status = nullptr;
  size_t lex_status_cap = 0;
  double* d_lex_scratch = nullptr;
  size_t lex_scratch_cap = 0;
  int32_t* d_redo_progs = nullptr;
  size_t redo_progs_cap = 0;
  // the exact pass (gpe_load_exact): programs re-evaluated with Python-int
  // semantics after every run of the loaded population
  int64_t n_exact = 0;
  int32_t* d_ex_progs = nullptr;
  size_t ex_progs_cap = 0;
  uint32_t* d_ex_code = nullptr;
  size_t ex_code_cap = 0;
  int64_t* d_ex_off = nullptr;
  size_t ex_off_cap = 0;
  uint32_t* d_ex_ints = nullptr;
  size_t ex_ints_cap = 0;
  double* d_ex_rows = nullptr;
  size_t ex_rows_cap = 0;
  // ... all of them as the host keeps them (gpe_load_exact_v): the device
  // list above holds those whose ints fit its 1088 bits; the host evaluates
  // the rest (ex_host), and every device program whose case outgrew them
  int64_t ex_all = 0;
  std::vector<int32_t> ex_h_progs;
  std::vector<uint32_t> ex_h_code;
  std::vector<int64_t> ex_h_off;
  std::vector<uint32_t> ex_h_words;     // int rows, variable length
  std::vector<int64_t> ex_h_woff;
  std::vector<int64_t> ex_dev_index;    // device list entry -> host entry
  std::vector<int64_t> ex_host;         // host entries never run on the device
  int64_t ex_host_runs = 0;             // programs the last run took to the host
  double ex_host_ms = 0.0;              // ... and the host pass's wall time
  uint64_t* d_exh_rec = nullptr;        // its results, scattered on the device
  size_t exh_rec_cap = 0;
  std::vector<double> ex_hX, ex_hT;     // the cases, copied back on first need
  bool ex_hcases = false;
  int cu = 0;
  int clock_khz = 0;
  char name[256] = {0};
  // multi-GPU: the RCCL communicator (gpe_comm_init) and its buffers
  ncclComm_t comm = nullptr;
  int comm_rank = 0, comm_world = 1;
  double* d_pair = nullptr;          // [2][n]: this rank's (hi, lo)
  size_t pair_cap = 0;
  double* d_gather = nullptr;        // [world][2][n] / [world][4][width]
  size_t gather_cap = 0;
  uint64_t* d_pack = nullptr;        // [4][width] (population sharding)
  size_t pack_cap = 0;
  uint8_t* d_tags = nullptr;         // caller tags gathered with the results
  size_t tags_cap = 0;
  int redo_global = 0;               // inside gpe_run_sharded*: redo flags
                                     // are combined over the ranks
};
