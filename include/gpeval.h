/*
 * gpeval.h — C ABI of the MI355X GP population evaluator (libgpeval.so).
 *
 * Drop-in boundary.  The reference evaluates a population with
 *     fitnesses = toolbox.map(toolbox.evaluate, invalid_ind)
 * (deap/algorithms.py:150,172), where every evaluate call runs
 * gp.compile (deap/gp.py:462-487) and a Python per-case loop
 * (examples/gp/symbreg.py:55-61, multiplexer.py:73-75, parity.py:66-68,
 * spambase.py:80-87).  deap_amd.evaluator replaces that map call by ONE
 * batched call into this library; the ctypes binding is
 * deap_amd/_lib.py.  Nothing here uses torch types: plain pointers/sizes.
 *
 * Conventions: functions return 0 on success or a negative GPE_E* code;
 * gpe_last_error() describes the last failure.  Host buffers are only read
 * during the call.  A context is bound to one device and is not thread-safe.
 * All entry points block until their work is complete.
 */
#ifndef GPEVAL_H
#define GPEVAL_H

#include <stddef.h>
#include <stdbool.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct gpe_ctx gpe_ctx;

/* machines (kernel families) */
#define GPE_MACHINE_F 0   /* fp64 accumulator machine: symreg, STGP */
#define GPE_MACHINE_B 1   /* bit-sliced boolean machine: mux, parity */

/* fitness modes */
#define GPE_MODE_MSE 0    /* sum over cases of (T - t0 - t1 - ...)^2, as a
                             double-double (hi, lo) pair; errors tracked   */
#define GPE_MODE_HITS_BOOL 1 /* F: count((T != 0) == (label != 0))        */
#define GPE_MODE_HITS_BITS 2 /* B: count(T == out) over bit-planes         */
#define GPE_MODE_SSE_NUMPY 3 /* F: sum over cases of (T - t0 - ...)^2 in
                                numpy.sum's exact order (pairwise over 8192-
                                element chunks); result in hi, lo = 0      */
#define GPE_MODE_SSE_SEQ 4   /* F: the same terms summed left to right from
                                0 (Python's builtin sum); hi, lo = 0       */

/* F-machine arithmetic (gpe_set_precision) */
#define GPE_PREC_F64 0    /* fp64 throughout: the reference's float        */
#define GPE_PREC_F32 1    /* fp32 cases/tree/d*d, fp64 double-double sum  */

/* error/flag encodings written by gpe_run */
#define GPE_NO_ERROR 0xFFFFFFFFFFFFFFFFull /* else (case << 2) | type       */
#define GPE_ERR_VALUE 1                    /* math.sin/cos(+-inf)          */
#define GPE_ERR_OVERFLOW 2                 /* (d)**2 overflow of finite d;
                                              exact pass: float(int) or
                                              int / int past 2**1024      */
#define GPE_ERR_XINT_RANGE 3               /* exact pass: an int past its
                                              1088-bit magnitude          */
#define GPE_XINT_WORDS 34                  /* uint32 words of an exact-pass
                                              int constant                */
#define GPE_FLAG_NONFINITE_TERM 1u         /* some d was inf or nan        */
#define GPE_FLAG_NAN_TERM 2u               /* some d*d was nan             */
#define GPE_FLAG_INF_TERM 4u               /* some d*d was +inf            */

#define GPE_E_INVALID -1
#define GPE_E_HIP -2
#define GPE_E_STATE -3
#define GPE_E_DEPTH -4
#define GPE_E_COMM -5       /* a collective did not complete within GPE_COMM_TIMEOUT_S */

/* Replaces: the per-process setup of the reference's evaluation
 * (nothing to bind on CPU; the device context owns streams/buffers). */
int gpe_create(int device, gpe_ctx** out);
void gpe_destroy(gpe_ctx* ctx);
const char* gpe_last_error(const gpe_ctx* ctx);
int gpe_device_info(const gpe_ctx* ctx, int* n_cu, int* clock_khz,
                    char* name, size_t name_len);

/* Upload the fitness cases once; they stay resident in HBM.
 * Replaces the case lists the reference's evaluate closes over
 * (symbreg.py:63 points, multiplexer.py:37-54 / parity.py:31-47 tables,
 * spambase.py:33-35 rows).
 *   F: X = double[n_vars][n_cases] (variable-planar), terms =
 *      double[n_terms][n_cases] (targets subtracted in order, or labels)
 *   B: X = uint32[n_vars][ceil(n_cases/32)] bit-planes (case c is bit c%32
 *      of word c/32), terms = uint32[ceil(n_cases/32)] output plane. */
int gpe_set_cases(gpe_ctx* ctx, int machine, const void* X, int n_vars,
                  int64_t n_cases, const void* terms, int n_terms);

/* Population-level evaluation of sin/cos leaves (F machine).  With
 * enable != 0 the context adds 2*n_vars columns, sin(x_v) then cos(x_v),
 * computed on the device at the start of every gpe_run with the same
 * near-correctly-rounded sin/cos as the interpreter; programs may then read
 * column n_vars + v for sin(ARGv) and 2*n_vars + v for cos(ARGv) (the
 * flattener's trig_leaves option).  Same values, one evaluation per case
 * instead of one per (program, case).  Must follow gpe_set_cases; discards
 * loaded programs. */
int gpe_set_trig_leaves(gpe_ctx* ctx, int enable);

/* Arithmetic of the F machine for the following runs (default GPE_PREC_F64).
 * GPE_PREC_F32 evaluates cases, constants, every node and (T - t)^2 in fp32
 * (device sinf/cosf), accumulating the squares in fp64 double-double: an
 * approximate throughput mode, not reference-exact (tolerance: DESIGN.md). */
int gpe_set_precision(gpe_ctx* ctx, int prec);

/* Upload one generation of flattened programs (deap_amd/flatten.py):
 * code = uint32 words, off[n_prog+1] word offsets, depth[n_prog] operand-
 * stack slots each program needs.  Replaces the n_prog gp.compile calls. */
int gpe_load_programs(gpe_ctx* ctx, const uint32_t* code, int64_t n_words,
                      const int64_t* off, int64_t n_prog,
                      const int32_t* depth);

/* Evaluate the loaded programs on the resident cases.  Outputs are HOST
 * arrays of n_prog entries (any may be NULL):
 *   out_hi/out_lo: MSE mode — double-double sum of squared errors;
 *                  hits modes — hit count in out_hi, 0 in out_lo
 *   out_err:       first erroring case per program (GPE_NO_ERROR if none)
 *   out_flags:     GPE_FLAG_* bits
 * Replaces: toolbox.map(toolbox.evaluate, invalid_ind) (algorithms.py:172)
 * minus the final division by len(points) and tuple packing. */
int gpe_run(gpe_ctx* ctx, int mode, double* out_hi, double* out_lo,
            uint64_t* out_err, uint32_t* out_flags);

/* Same, but writing DEVICE arrays (e.g. torch tensors) so that the caller
 * can all-reduce partial sums over RCCL before copying to the host. */
int gpe_run_device(gpe_ctx* ctx, int mode, void* d_hi, void* d_lo,
                   void* d_err, void* d_flags);

/* gpe_run plus the per-case terms behind the reduction, for selection
 * schemes that need them (lexicase: reference deap/tools/selection.py:
 * 214-320 reads one fitness value per case).  out_cases is a HOST array
 * double[n_prog][n_cases]: MSE mode — (T - t0 - ...)^2 per case, exactly the
 * values the SSE sums; HITS_BOOL — 1.0 for a hit, 0.0 otherwise.  F machine
 * only; the other outputs are those of gpe_run. */
int gpe_run_cases(gpe_ctx* ctx, int mode, double* out_cases, double* out_hi,
                  double* out_lo, uint64_t* out_err, uint32_t* out_flags);

/* Device lexicase selection that replays the reference's random stream:
 * selLexicase (mode 0), selEpsilonLexicase (mode 1, epsilon) and
 * selAutomaticEpsilonLexicase (mode 2; n <= 16384) of deap/tools/
 * selection.py:214-320.  values is a HOST double[n][n_cases]
 * (fitness.values per individual), or NULL to select on the per-case
 * matrix of the last gpe_run_cases (n = programs) without a host round
 * trip.  maximise[n_cases]: 1 where the case's weight is positive.
 * mt_state[625] (in/out): CPython's MT19937 state as random.getstate()[1]
 * gives it (624 words, then the position); the kernel makes the
 * reference's draws — random.shuffle(cases), then random.choice(candidates),
 * per selection — and writes back the state after them (random.setstate).
 * Writes the k selected indices.  *failed = -1, or the index of the
 * selection that ended with no candidate (where the reference raises
 * IndexError from random.choice([])); out and mt_state then stop there. */
int gpe_lexicase(gpe_ctx* ctx, const double* values, int64_t n,
                 int64_t n_cases, const uint8_t* maximise, int mode,
                 double epsilon, uint32_t* mt_state, int64_t k, int32_t* out,
                 int64_t* failed);

/* Device tournament selection that replays the reference's random stream:
 * selTournament (deap/tools/selection.py:51-69, aspirants drawn by selRandom
 * :15-28, i.e. random.choice) — k tournaments of tournsize aspirants, the
 * winner the first aspirant with the greatest fitness (Fitness.__gt__:
 * not (a.wvalues <= b.wvalues), Python tuple order).  wvalues is a HOST
 * double[n][nobj] (fitness.wvalues per individual), or NULL to select on the
 * last gpe_run's fitness still on the device (MSE: (hi + lo) / n_cases,
 * SSE and hit modes: hi), times `weight` (nobj = 1, n = programs) — no host
 * round trip.  mt_state[625] (in/out) as in gpe_lexicase: the draws are
 * CPython's getrandbits rejection sampling on MT19937, and the state after
 * them is written back.  Writes the k selected indices to out. */
int gpe_tournament(gpe_ctx* ctx, const double* wvalues, int64_t n, int nobj,
                   double weight, int64_t k, int tournsize, uint32_t* mt_state,
                   int32_t* out);

/* ---- Lowering on the device (the host flattener's job, deap_amd/flatten.py
 * Flattener._build/_emit/_encode, run one tree per GPU thread from the same
 * source, deap_amd/csrc/lower_core.h).  The host maps each node object of a
 * PrimitiveTree (reference deap/gp.py:44-184) to an entry of the primitive
 * set (deap/gp.py:260-456) and uploads one byte per node. */
typedef struct {          /* a Python number as the constant fold sees it */
  char t;                 /* 'f' float, 'i' int, 'b' bool, 'x' unsupported */
  double f;
  int64_t i;
  bool err_value;         /* the fold raised ValueError (sin/cos of inf) */
} gpe_value;
typedef struct {          /* one primitive / terminal of the pset */
  int32_t kind;           /* 0 primitive, 1 argument, 2 constant terminal */
  int32_t arity;
  int32_t sem;            /* deap_amd/flatten.py _NATIVE_SEM */
  int32_t var;            /* argument index */
  gpe_value c;            /* constant terminal's value */
} gpe_entry;

/* The pset tables of gpe_lower_programs: the machine (GPE_MACHINE_*), the
 * number of case variables, per argument whether sin/cos of it is read from
 * a trig-leaf column (gpe_set_trig_leaves), and the entries (< 255). */
int gpe_set_lowering(gpe_ctx* ctx, int machine, int nv, const uint8_t* leaf,
                     int n_leaf, const gpe_entry* entries, int n_entries);

/* Lower n trees on the device and load them as programs (as
 * gpe_load_programs does with host-flattened words).  codes[node_off[i] ..
 * node_off[i+1]) are tree i's node entries in prefix order, 255 for an
 * ephemeral constant whose value is the next of evals[eph_off[i] ..
 * eph_off[i+1]).  Per tree (host arrays): out_depth, out_err (0, 3 =
 * SyntaxError of a too-tall tree, 4 = a raising constant fold), out_status
 * (bit 0: declined — the host flattener must lower it, Python semantics the
 * device fold does not cover; bit 1: an int constant beyond 2^53 evaluated
 * in float64; bit 2: the raising fold is ValueError).  A declined tree is
 * loaded as END; the caller re-flattens the batch on the host.  On an error
 * return the context holds no programs.  Trees past 65,535 nodes are
 * declined (the device's lowering records hold 16-bit node indices). */
int gpe_lower_programs(gpe_ctx* ctx, const uint8_t* codes, const int64_t* node_off,
                       int64_t n, const gpe_value* evals, const int64_t* eph_off,
                       int32_t* out_depth, uint8_t* out_err, uint8_t* out_status);

/* gpe_lower_programs in chunks, for callers that read the trees in chunks:
 * the same result as one call on the concatenated trees, but each chunk's
 * upload and lowering run on the device (asynchronously, on the context's
 * stream) while the caller reads the next one.  gpe_lower_begin(n_total),
 * then gpe_lower_add for consecutive chunks of the trees (each chunk's
 * node_off / eph_off start at 0; its arrays may be freed when the call
 * returns), then gpe_lower_end with the per-tree outputs of all n_total
 * trees.  No other call may use the context in between; an error ends the
 * lowering (the context then holds no programs).  GPUEvaluator reads a
 * million trees in chunks (deap_amd/evaluator.py lower_on_device). */
int gpe_lower_begin(gpe_ctx* ctx, int64_t n_total);
/* gpe_lower_begin with the per-tree outputs given up front (all n_total
 * entries; they must stay valid until gpe_lower_end): each gpe_lower_add
 * then decodes the chunks whose metadata has reached the host, on the
 * caller's thread, so that gpe_lower_end is left with the last chunks only.
 * gpe_lower_end is then called with these pointers or with NULLs. */
int gpe_lower_begin_into(gpe_ctx* ctx, int64_t n_total, int32_t* out_depth, uint8_t* out_err,
                         uint8_t* out_status);
int gpe_lower_add(gpe_ctx* ctx, const uint8_t* codes, const int64_t* node_off, int64_t n,
                  const gpe_value* evals, const int64_t* eph_off);
int gpe_lower_end(gpe_ctx* ctx, int32_t* out_depth, uint8_t* out_err, uint8_t* out_status);
/* After gpe_lower_end (or gpe_lower_programs): how many of the trees got a
 * nonzero error code / status, so that a caller can skip scanning a million
 * zeros. */
int gpe_last_lower_flags(gpe_ctx* ctx, int64_t* n_err, int64_t* n_status);

/* gpe_load_programs + gpe_run. */
int gpe_eval(gpe_ctx* ctx, int mode, const uint32_t* code, int64_t n_words,
             const int64_t* off, int64_t n_prog, const int32_t* depth,
             double* out_hi, double* out_lo, uint64_t* out_err,
             uint32_t* out_flags);

/* Exact-integer pass.  The reference evaluates trees with Python numbers
 * (gp.compile, deap/gp.py:462-487): int constants (rand101,
 * examples/gp/symbreg.py:43) and protectedDiv's int 1 (:29-33) stay exact
 * ints through operator.add/sub/mul/neg, int / int rounds the exact ratio
 * once, and ints compare exactly with floats.  The kernels compute in
 * float64, which agrees while every int stays within 2^53.  The n programs
 * listed here (flatten.py Flattener.exact_programs: those whose ints can
 * pass 2^53) are re-evaluated after every run of the loaded population
 * with Python's semantics (glibc sin/cos), overwriting their outputs: hi/lo
 * and the per-case matrix of gpe_run_cases.  The device holds ints as sign
 * + 1088-bit magnitude; a program with a wider int constant, and a device
 * program whose case outgrew 1088 bits, is evaluated on the host with
 * unbounded ints instead (the same semantics, the same order of summation),
 * so every result is the reference's.  Modes MSE, SSE_SEQ (the exact pass
 * sums in its fixed order) and HITS_BOOL, fp64 only; SSE_NUMPY and fp32 runs
 * skip the pass.  A case's first exception goes to out_err as the reference
 * raises it: GPE_ERR_VALUE (sin/cos(inf)), GPE_ERR_OVERFLOW (float(int) or
 * int / int past the float range, or d**2).
 * progs[n]: indices into the loaded population; code/off/depth: their
 * programs in the usual words, except that an int constant has index field
 * 1 and its row of the int table in its two data words (low word first).
 * The table: n_ints rows of little-endian 32-bit words in two's complement,
 * row r = int_words[int_off[r] .. int_off[r + 1]) (int_off[0] = 0).
 * Cleared by gpe_load_programs, gpe_lower_programs and gpe_set_cases (call
 * it after those); n = 0 clears. */
int gpe_load_exact_v(gpe_ctx* ctx, const int32_t* progs, int64_t n,
                     const uint32_t* code, int64_t n_words, const int64_t* off,
                     const int32_t* depth, const uint32_t* int_words,
                     const int64_t* int_off, int64_t n_ints);

/* gpe_load_exact_v with rows of GPE_XINT_WORDS words: ints[n_ints][34],
 * and the round-4 encoding of an int constant (index field 1 + row, the
 * f64 bits in its data words), translated to gpe_load_exact_v's. */
int gpe_load_exact(gpe_ctx* ctx, const int32_t* progs, int64_t n,
                   const uint32_t* code, int64_t n_words, const int64_t* off,
                   const int32_t* depth, const uint32_t* ints, int64_t n_ints);

/* Exact-pass programs the last run evaluated on the host (ints past the
 * device's 1088 bits). */
int gpe_last_exact_host_runs(gpe_ctx* ctx, int64_t* n);

/* ... and the wall time of that host pass, ms (0 when none ran): a slow
 * host fallback shows up in the caller's stats. */
int gpe_last_exact_host_ms(gpe_ctx* ctx, double* ms);

/* ---- Multi-GPU over one node: one process per GPU,
 * each with its own context; the context owns an RCCL communicator.
 * Replaces the reference's only parallelism, a user-registered
 * multiprocessing.Pool.map over individuals (examples/ga/onemax_mp.py:58-59,
 * doc/tutorials/basic/part4.rst:19-56), which has no C-level interface.
 * RCCL is opened at first use (dlopen librccl.so.1); GPE_E_STATE if absent. */
#define GPE_UNIQUE_ID_BYTES 128

/* Rank 0 creates the communicator id (ncclGetUniqueId) and hands the
 * GPE_UNIQUE_ID_BYTES bytes to the other ranks by any means (a file, a
 * socket, torch.distributed's broadcast); no context needed. */
int gpe_comm_unique_id(void* id_out);

/* Join the communicator (ncclCommInitRank on the context's device).
 * Collective: every rank calls it with the same id and world. */
int gpe_comm_init(gpe_ctx* ctx, int rank, int world, const void* unique_id);

/* rank / world of the context's communicator (-1 / 0 if none). */
int gpe_comm_info(const gpe_ctx* ctx, int* rank, int* world);

/* Case sharding (config 4): this rank holds cases [case_offset,
 * case_offset + n_cases) (gpe_set_cases) and the same programs as every
 * rank.  gpe_run on the slice, then on the context's stream: the (hi, lo)
 * partials are all-gathered and summed in rank order as double-doubles, the
 * first-error codes (global case index) reduced with MIN and the flag bits
 * OR-ed.  Every rank receives the whole-population result.  MSE and hits
 * modes only (GPE_E_INVALID for the order-exact numpy / builtin-sum modes).
 * Collective.  _device: outputs are device arrays (NULL: the context's own),
 * no host synchronisation; otherwise host arrays of n_prog entries. */
int gpe_run_sharded_device(gpe_ctx* ctx, int mode, int64_t case_offset,
                           void* d_hi, void* d_lo, void* d_err, void* d_flags);
int gpe_run_sharded(gpe_ctx* ctx, int mode, int64_t case_offset,
                    double* out_hi, double* out_lo, uint64_t* out_err,
                    uint32_t* out_flags);

/* Population sharding (config 3): each rank loaded its own slice of the
 * programs (at most `width`); after gpe_run they are all-gathered, so every
 * rank receives host arrays of world * width entries, rank r's program i at
 * r * width + i (entries past a rank's n_prog: hi = lo = 0, err =
 * GPE_NO_ERROR, flags = 0).  tags (n_prog bytes, may be NULL) travel with
 * the results in bits 8..15 of out_flags (the Python layer sends the
 * flattener's per-tree verdicts this way).  Collective. */
int gpe_run_gathered(gpe_ctx* ctx, int mode, int64_t width,
                     const uint8_t* tags, double* out_hi, double* out_lo,
                     uint64_t* out_err, uint32_t* out_flags);

/* Device time of the last gpe_run* (HIP events on the context's stream):
 * ms[0] = interpreter kernels, ms[1] = reduction kernel, ms[2] = total. */
int gpe_last_timing(const gpe_ctx* ctx, float* ms);

/* Collective time of the last sharded run (HIP events on the context's
 * stream): ms[0] = the RCCL group of gpe_run_sharded* (all-gather of the
 * partials, first-error MIN, flag SUM) or the all-gather of
 * gpe_run_gathered, ms[1] = the case-sharded redo-flag all-reduce (0 when
 * none ran: the exact cores raise no flags).  Every wait on a stream that
 * holds collectives is bounded by GPE_COMM_TIMEOUT_S seconds (default 120):
 * past it the communicator is aborted and the call returns GPE_E_COMM with
 * the collective, rank and RCCL's asynchronous error in gpe_last_error().
 * Replaces nothing in the reference (its Pool.map, examples/ga/
 * onemax_mp.py:58-59, has no collectives to time or bound). */
int gpe_last_comm_timing(gpe_ctx* ctx, float* ms);

/* Test infrastructure (no HIP calls): the bounded wait above on a fake
 * stream that stays busy for `busy_polls` queries (< 0: forever); returns
 * 0 or GPE_E_COMM and the message a timed-out collective would report. */
int gpe_debug_bounded_wait(double timeout_s, int64_t busy_polls, char* msg, size_t n);

/* Launch geometry of the last gpe_run (for reports): programs on the asm
 * core, on the C++ fast and deep kernels, programs re-run because a sin/cos
 * argument left the asm core's range, programs per wave, tile groups,
 * (program, tile) pairs that raised the re-run flag, waves per block. */
int gpe_last_geometry(const gpe_ctx* ctx, int64_t* out8);

/* gpe_last_geometry's eight fields (there "programs on the asm core" counts
 * both asm cores), then for the deep asm core (programs needing 6..12 stack
 * slots): programs, programs per wave, tile groups, waves per block; then
 * the re-run programs that the exact asm core (glibc's sin/cos) left to the
 * C++ exact kernels (a sin/cos argument at or past 105414350, inf or nan);
 * then for the typed asm core (GPE_MODE_HITS_BOOL: PrimitiveSetTyped
 * programs, spambase.py): programs, programs per wave, tile groups; then
 * the HITS_BOOL programs that are one folded constant, whose hit count
 * (the cases whose label has the constant's truth) needs no core run.
 * Writes the first min(n, GPE_GEOMETRY_FIELDS) fields. */
#define GPE_GEOMETRY_FIELDS 17
int gpe_last_geometry_ex(const gpe_ctx* ctx, int64_t* out, int n);

/* Diagnostic (host only): the program -> threaded-code translation the asm
 * core executes, with a caller-given handler table; starts[i] = -1 for
 * programs the asm core does not run.  Lets CPU tests check translation and
 * jump targets without a GPU. */
int gpe_debug_translate(const uint32_t* code, int64_t n_words,
                        const int64_t* off, int64_t n_prog,
                        const int32_t* depth, int nv, const uint32_t* table,
                        int n_table, uint32_t* out, int64_t out_cap,
                        int64_t* starts, int64_t* n_out);

/* Diagnostic: evaluate the device's sin (fn 0), cos (fn 1), square (fn 2),
 * the platform libm's sin (3) / cos (4), or sin (5) / cos (6) through the
 * hand-scheduled asm interpreter core; fp32 mode: sin (7) / cos (8) through
 * the fp32 asm core, sin (9) / cos (10) of the C++ kernels; glibc_sin (11) /
 * glibc_cos (12), the restatement of the reference's libm; sin (13) /
 * cos (14) through the exact asm core (glibc's algorithm in the handler;
 * arguments it leaves to the C++ pass through glibc_sin/cos); on n host
 * inputs — the elementary operations whose rounding can differ from glibc.
 * Used by the parity tests to quantify ulp differences. */
int gpe_math_probe(gpe_ctx* ctx, int fn, const double* x, double* y,
                   int64_t n);

/* The same sin (0) / cos (1) / square (2) code compiled for the host CPU
 * (no GPU needed): lets the CPU test suite check the kernels' elementary
 * functions bit for bit against correctly rounded values.  3 / 4: the fp32
 * mode's sin / cos of (float)x, returned as double.  5 / 6: glibc_sin /
 * glibc_cos (the restatement of glibc 2.35's sin/cos the redo pass uses;
 * checked against the host libm bit for bit).  7 / 8: the same through the
 * exact interpreter's two-cases-at-once form (glibc_trig_k). */
int gpe_host_math(int fn, const double* x, double* y, int64_t n);

/* Host twin of the GPE_MODE_SSE_NUMPY reduction (test infrastructure): the
 * numpy.sum of each of n_rows contiguous rows of n_cols doubles, in
 * numpy's order (replaces numpy.sum at examples/gp/symbreg_numpy.py:66). */
int gpe_host_np_sum(const double* x, int64_t n_rows, int64_t n_cols,
                    double* out);

/* Test infrastructure for the multi-rank collectives on one device.
 * gpe_debug_shard_combine: gpe_run_sharded_device's combine for `world`
 * ranks whose outputs the caller gives (parts[world][2][n]: each rank's
 * (hi, lo) partials, the buffer its RCCL all-gather fills; errs[world][n],
 * flags[world][n]: each rank's first-error words and flag bits as its run
 * left them; case_offsets[world]): the same shard_prep and shard_finish
 * kernels, with the two all-reduces (MIN of the errors, SUM of the packed
 * flag counters) computed on the device from the given arrays.  Replaces
 * the reference's Pool.map over individuals
 * (examples/ga/onemax_mp.py:58-59), which has no combine of its own.
 * gpe_debug_redo_union: redo flags (one per loaded program, n = 0 clears)
 * that "other ranks" raised; every later run ORs them into this context's
 * own before its redo pass, as the case-sharded all-reduce (MAX) does. */
int gpe_debug_shard_combine(gpe_ctx* ctx, int world, int64_t n,
                            const double* parts, const uint64_t* errs,
                            const uint32_t* flags, const int64_t* case_offsets,
                            double* out_hi, double* out_lo, uint64_t* out_err,
                            uint32_t* out_flags);
int gpe_debug_redo_union(gpe_ctx* ctx, const uint32_t* flags, int64_t n);

/* Host twin of the exact pass's device interpreter (test infrastructure):
 * one program (gpe_load_exact_v's encoding and int table) on one case
 * x[nv].  Returns 0, the case's GPE_ERR_* (1 ValueError, 2 OverflowError,
 * 3 past the device's 1088 bits), or a negative error.  *out_isint: whether
 * the result is a Python int; *out_f: float(result) (inf where that would
 * overflow); out_words[GPE_XINT_WORDS]: the int as 1088-bit two's
 * complement. */
int gpe_host_exact_eval(const uint32_t* code, const uint32_t* int_words,
                        const int64_t* int_off, int64_t n_ints, const double* x,
                        int nv, double* out_f, uint32_t* out_words, int* out_isint);

/* The host evaluator of the exact pass's wide programs (no int size limit;
 * csrc/bigint_host.h) on one case.  Returns as gpe_host_exact_eval, never
 * 3.  The int result goes to out_words as two's complement in
 * *inout_nwords words (the capacity in, the count out; a capacity too small
 * returns GPE_E_INVALID with the count needed; out_words NULL: the count
 * only). */
int gpe_host_bigint_eval(const uint32_t* code, const uint32_t* int_words,
                         const int64_t* int_off, int64_t n_ints, const double* x,
                         int nv, double* out_f, uint32_t* out_words,
                         int64_t* inout_nwords, int* out_isint);

#ifdef __cplusplus
}
#endif

#endif /* GPEVAL_H */
