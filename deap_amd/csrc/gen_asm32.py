#!/usr/bin/env python3
"""Generate the fp32 interpreter core (``gp_asm_core32.inc``) of the fp32
mode (``gpe_set_precision(GPE_PREC_F32)``).

Same threaded-code design as ``gen_asm.py`` (SGPR program window, handlers
specialised by stack slot and variable, the same handler list and therefore
the same handler-id layout, so the host translator serves both cores), with
fp32 values: T, the operand stack and the LDS case tile hold one float per
case, K = 4 cases per lane.  Inline constants arrive as fp32 bits in the
first of their two program words (host translation).

sin/cos (``gp_trig32`` in gpeval.hip, operation for operation): x = k*pi/2 + r
with k = rint(x * 2/pi), r by a three-part Cody-Waite reduction with FMA
(|x| < 2^30), then the sin and cos polynomials of r (cephes sinf/cosf
coefficients on [-pi/4, pi/4]) selected and signed by the quadrant.

Per case k the core keeps in VRED_k the running unsigned min of
``key(x) = 2|x|.bits - 2 LIM  (mod 2^32)`` over its sin/cos arguments — one
``v_lshl_add_u32`` (the sign bit shifts out) and one ``v_min_u32``.  The key
orders the argument classes as

    finite >= 2^30  <  +-inf (== RED_INF)  <  nan  <  finite < 2^30

so after the program: VRED_k < RED_INF — a finite argument reached 2^30 and
the core's result is not usable: the (program, tile) pair is re-run on the
C++ kernels; == RED_INF — no such argument, an infinite one: ValueError, as
the reference's math.sin raises (fp32 overflows to inf far more often than
fp64, so this is decided here rather than re-run); anything else — every
reduction was exact (nan arguments propagate nan, as math.sin does).

Register contract:
    v[TB0 : TB0+K)       T  accumulator, K floats
    v[RB : RB+KD)        R  operand stack, slot d case k at RB + dK + k
    VRED_k (K regs)      per case: max |x| bits of its sin/cos arguments
    VS2, VC2             the polynomial constants S2, C2 (VOP3 operands)
    temporaries          generator-allocated; division temps and O share it
    s[SB : SB+16)        program window
    s[SB+16 : SB+32)     constants INV, P1, P2, P3, S1, S2, S3, C1, C2, C3
    (remaining SGPRs as in gen_asm.py)
"""
import os
import struct
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import gen_asm  # noqa: E402
from gen_asm import FAMS, WINDOW  # noqa: E402

LIM32 = 0x4e800000                  # bits of 2^30 (f32)
INF32 = 0x7f800000
RED_BIAS = (-2 * LIM32) & 0xffffffff     # key(x) = 2|x|.bits + RED_BIAS
RED_INF = (2 * INF32 + RED_BIAS) & 0xffffffff   # key(+-inf)
# (name, value) in SGPR order; values are exactly representable in f32
CONSTS = [("INV", 0.6366197466850281), ("P1", 1.5707963705062866),
          ("P2", -4.371138828673793e-08), ("P3", -1.7151245100058819e-15),
          ("S1", -1.6666654611e-1), ("S2", 8.3321608736e-3),
          ("S3", -1.9515295891e-4), ("C1", 4.166664568298827e-2),
          ("C2", -1.388731625493765e-3), ("C3", 2.443315711809948e-5),
          # not a number used as one: the bit pattern RED_BIAS (an SGPR
          # operand of the key computation; VOP3 takes no literal on gfx950)
          ("RED", struct.unpack("<f", struct.pack("<I", RED_BIAS))[0])]


def f32bits(v):
    return struct.unpack("<I", struct.pack("<f", v))[0]


def f32(v):
    return struct.unpack("<f", struct.pack("<f", v))[0]


class Gen32(gen_asm.Gen):
    def __init__(self, K, D, NV, TB0=32, SB=56):
        # wave priority (GEN_ASM32_PRIO, default "tiered"; "none": no
        # s_setprio): light handlers 2, protectedDiv 1, sin/cos 0, as
        # gen_asm.py's cores (same-box fp32 leg 348.5 -> 328.3 ms)
        self.prio = (2, 0, 1) if os.environ.get("GEN_ASM32_PRIO", "tiered") == "tiered" else None
        self.K, self.D, self.NV = K, D, NV
        self.TB0 = TB0
        self.RB = TB0 + K
        self.VRED = self.RB + K * D
        self.VS2 = self.VRED + K
        self.VC2 = self.VRED + K + 1
        self.POOL0 = self.VRED + K + 2
        # division temporaries (5) then the operand scratch O (K)
        self.OB = self.POOL0 + 6
        self.vmax = self.OB + K
        assert SB % 4 == 0
        self.SB = SB
        self.WIN = SB
        self.TC = SB + 16
        self.BASE = SB + 32
        self.PTR = SB + 34
        self.TGT = SB + 36
        self.CA = SB + 38
        self.NXT = SB + 40
        self.SM0 = SB + 41
        self.SMAX = SB + 41
        self.lines = []
        self.handlers = []
        self.align = 0                 # handlers packed (gen_asm.Gen.handler)
        self.loop = self.typed = False  # per-program core, fp64 families
        self.fams = gen_asm.FAMS

    # registers: one VGPR per value
    @staticmethod
    def p(n):
        return "v%d" % n

    def T(self, k):
        return self.TB0 + k

    def R(self, d, k):
        return self.RB + d * self.K + k

    def O(self, k):
        return self.OB + k

    def sc(self, name):
        return "s%d" % (self.TC + [n for n, _ in CONSTS].index(name))

    # ------------------------------------------------------- arithmetic --
    def ldx(self, dst_base, v):
        for k in range(self.K):
            self.e("ds_read_b32 v%d, %%[xa] offset:%d"
                   % (dst_base + k, (v * self.K + k) * 256))

    def division(self, q, num, den, tmp):
        """q = num / den (IEEE fp32, the compiler's gfx950 sequence)."""
        a, b, c, dd, e = tmp
        self.e("v_div_scale_f32 v%d, vcc, %s, %s, %s" % (a, den, den, num))
        self.e("v_rcp_f32_e32 v%d, v%d" % (b, a))
        self.e("v_div_scale_f32 v%d, vcc, %s, %s, %s" % (c, num, den, num))
        self.e("v_fma_f32 v%d, -v%d, v%d, 1.0" % (dd, a, b))
        self.e("v_fmac_f32_e32 v%d, v%d, v%d" % (b, dd, b))
        self.e("v_mul_f32_e32 v%d, v%d, v%d" % (dd, c, b))
        self.e("v_fma_f32 v%d, -v%d, v%d, v%d" % (e, a, dd, c))
        self.e("v_fmac_f32_e32 v%d, v%d, v%d" % (dd, e, b))
        self.e("v_fma_f32 v%d, -v%d, v%d, v%d" % (a, a, dd, c))
        self.e("v_div_fmas_f32 v%d, v%d, v%d, v%d" % (a, a, b, dd))
        self.e("v_div_fixup_f32 v%d, v%d, %s, %s" % (q, a, den, num))

    def _div_common(self, k, num, den):
        tmp = [self.POOL0 + i for i in range(5)]
        q = self.POOL0 + 5
        self.use_v(q)
        self.division(q, num, den, tmp)
        return q, tmp

    def pdiv(self, k, num, den):
        """T_k = (den == 0) ? 1.0 : num / den   (protectedDiv)."""
        q, tmp = self._div_common(k, num, den)
        self.e("v_cmp_neq_f32_e64 vcc, 0, %s" % den)   # nan: keeps q
        self.e("v_cndmask_b32_e32 v%d, 1.0, v%d, vcc" % (self.T(k), q))

    def npdiv(self, k, num, den):
        """T_k = num / den, inf or nan -> 1.0 (symbreg_numpy.py:28-36)."""
        q, tmp = self._div_common(k, num, den)
        self.e("s_movk_i32 s%d, 0x1f8" % self.NXT)      # finite classes
        self.e("v_cmp_class_f32_e64 vcc, v%d, s%d" % (q, self.NXT))
        self.e("v_cndmask_b32_e32 v%d, 1.0, v%d, vcc" % (self.T(k), q))

    def binops(self, fam, operands):
        """binop() for every case; protectedDiv bodies at the middle priority."""
        tier = self.prio is not None and fam in ("div", "rdiv", "ndiv", "nrdiv")
        if tier:
            self.e("s_setprio %d" % self.prio[2])
        for k in range(self.K):
            self.binop(fam, k, operands[k])
        if tier:
            self.e("s_setprio %d" % self.prio[0])

    def binop(self, fam, k, a):
        T = "v%d" % self.T(k)
        if fam == "add":
            self.e("v_add_f32_e32 %s, %s, %s" % (T, a, T))
        elif fam == "sub":
            self.e("v_sub_f32_e32 %s, %s, %s" % (T, a, T))
        elif fam == "rsub":
            self.e("v_subrev_f32_e32 %s, %s, %s" % (T, a, T))
        elif fam == "mul":
            self.e("v_mul_f32_e32 %s, %s, %s" % (T, a, T))
        elif fam == "div":
            self.pdiv(k, a, T)
        elif fam == "rdiv":
            self.pdiv(k, T, a)
        elif fam == "ndiv":
            self.npdiv(k, a, T)
        elif fam == "nrdiv":
            self.npdiv(k, T, a)
        else:
            raise KeyError(fam)

    # ---------------------------------------------------------- sin/cos --
    def trig_ops32(self, k, want):
        """gp_trig32() for case k: (template, defs, uses); all singles."""
        c = self.sc
        ops = []

        def op(t, d=(), u=()):
            ops.append((t, tuple(d), tuple(u)))
        op("v_lshl_add_u32 {ax}, {x}, 1, %s" % c("RED"), ["ax"], ["x"])
        op("v_min_u32_e32 v%d, v%d, {ax}" % (self.VRED + k, self.VRED + k),
           [], ["ax"])
        op("v_mul_f32_e32 {p}, %s, {x}" % c("INV"), ["p"], ["x"])
        op("v_rndne_f32_e32 {kf}, {p}", ["kf"], ["p"])
        op("v_fma_f32 {r}, -{kf}, %s, {x}" % c("P1"), ["r"], ["kf", "x"])
        op("v_fma_f32 {r}, -{kf}, %s, {r}" % c("P2"), ["r"], ["kf", "r"])
        op("v_fma_f32 {r}, -{kf}, %s, {r}" % c("P3"), ["r"], ["kf", "r"])
        op("v_cvt_i32_f32_e32 {q}, {kf}", ["q"], ["kf"])
        if want == "cos":
            op("v_add_u32_e32 {q}, 1, {q}", ["q"], ["q"])
        op("v_mul_f32_e32 {z}, {r}, {r}", ["z"], ["r"])
        op("v_fma_f32 {ps}, {z}, %s, v%d" % (c("S3"), self.VS2), ["ps"],
           ["z"])
        op("v_fmaak_f32 {ps}, {ps}, {z}, 0x%08x" % f32bits(CONSTS[4][1]),
           ["ps"], ["ps", "z"])
        op("v_mul_f32_e32 {rz}, {r}, {z}", ["rz"], ["r", "z"])
        op("v_fma_f32 {s}, {rz}, {ps}, {r}", ["s"], ["rz", "ps", "r"])
        op("v_fma_f32 {pc}, {z}, %s, v%d" % (c("C3"), self.VC2), ["pc"],
           ["z"])
        op("v_fmaak_f32 {pc}, {pc}, {z}, 0x%08x" % f32bits(CONSTS[7][1]),
           ["pc"], ["pc", "z"])
        op("v_fma_f32 {c0}, {z}, -0.5, 1.0", ["c0"], ["z"])
        op("v_mul_f32_e32 {z2}, {z}, {z}", ["z2"], ["z"])
        op("v_fma_f32 {cc}, {z2}, {pc}, {c0}", ["cc"], ["z2", "pc", "c0"])
        op("v_and_b32_e32 {t}, 1, {q}\n"
           "v_cmp_ne_u32_e32 vcc, 0, {t}\n"
           "v_cndmask_b32_e32 {res}, {s}, {cc}, vcc",
           ["t", "res"], ["q", "s", "cc"])
        op("v_lshlrev_b32_e32 {sg}, 30, {q}", ["sg"], ["q"])
        op("v_and_b32_e32 {sg}, 0x80000000, {sg}", ["sg"], ["sg"])
        op("v_xor_b32_e32 {x}, {res}, {sg}", [], ["res", "sg"])
        return ops

    def sincos(self, want):
        """The K chains interleaved op by op; temporaries linear-scan
        allocated (single VGPRs) from the pool."""
        K = self.K
        chains = [self.trig_ops32(k, want) for k in range(K)]
        seq = [(k,) + chains[k][i] for i in range(len(chains[0]))
               for k in range(K)]
        last = {}
        for idx, (k, t, d, u) in enumerate(seq):
            for v in u:
                last[(k, v)] = idx
        for idx, (k, t, d, u) in enumerate(seq):
            for v in d:
                last.setdefault((k, v), idx)
        free, nxt, where = [], [self.POOL0], {}

        def get():
            if free:
                return free.pop(0)
            r = nxt[0]
            nxt[0] += 1
            return r

        for idx, (k, t, d, u) in enumerate(seq):
            multi = "\n" in t
            names = {"x": "v%d" % self.T(k)}
            for v in u:
                if v != "x":
                    names[v] = "v%d" % where[(k, v)]
            dying = [v for v in set(u) if v != "x" and last[(k, v)] == idx]
            if not multi:
                for v in dying:
                    free.append(where.pop((k, v)))
                free.sort()
            for v in d:
                if (k, v) not in where:
                    where[(k, v)] = get()
                names[v] = "v%d" % where[(k, v)]
            if multi:
                for v in dying:
                    free.append(where.pop((k, v)))
                free.sort()
            for line in t.split("\n"):
                self.e(line.format(**names))
            for v in d:
                if (k, v) in where and last[(k, v)] == idx:
                    free.append(where.pop((k, v)))
                    free.sort()
        self.use_v(nxt[0] - 1)

    # ----------------------------------------------------------- build --
    def build(self):
        K, D, NV = self.K, self.D, self.NV
        W, TC = self.WIN, self.TC
        self.e("s_mov_b32 s%d, m0" % self.SM0)
        self.prologue_base()
        if self.prio:
            self.e("s_setprio %d" % self.prio[0])
        self.e("s_mov_b64 %s, %%[pc]" % self.sp(self.PTR))
        for k in range(K):
            self.e("v_mov_b32_e32 v%d, -1" % (self.VRED + k))
        self.e("s_cmp_eq_u32 %[probe], 0")
        self.e("s_cbranch_scc1 .Lrun_%=")
        self.e("s_branch .Lprobe_%=")
        self.label(".Lrun_")
        self.e("s_load_dwordx16 s[%d:%d], %%[cst], 0x0" % (TC, TC + 15))
        self.e("s_load_dwordx16 s[%d:%d], %s, 0x0"
               % (W, W + 15, self.sp(self.PTR)))
        self.e("s_mov_b32 m0, 0")
        self.e("s_waitcnt lgkmcnt(0)")
        self.e("v_mov_b32_e32 v%d, %s" % (self.VS2, self.sc("S2")))
        self.e("v_mov_b32_e32 v%d, %s" % (self.VC2, self.sc("C2")))
        self.dispatch_head()
        self.dispatch_tail()
        self.handler("END")
        self.e("s_branch .Lend_%=")
        self.handler("RELOAD")
        self.e("s_add_u32 s%d, s%d, %d" % (self.PTR, self.PTR, 4 * WINDOW))
        self.e("s_addc_u32 s%d, s%d, 0" % (self.PTR + 1, self.PTR + 1))
        self.e("s_load_dwordx16 s[%d:%d], %s, 0x0"
               % (W, W + 15, self.sp(self.PTR)))
        self.e("s_mov_b32 m0, 0")
        self.e("s_waitcnt lgkmcnt(0)")
        self.e("s_nop 0")
        self.dispatch_head()
        self.dispatch_tail()
        CA = "s%d" % self.CA
        self.handler("LDC")
        self.dispatch_head(2)
        for k in range(K):
            self.e("v_mov_b32_e32 v%d, %s" % (self.T(k), CA))
        self.dispatch_tail()
        for v in range(NV):
            self.handler("LDV%d" % v)
            self.ldx(self.T(0), v)
            self.dispatch_head()
            self.e("s_waitcnt lgkmcnt(0)")
            self.dispatch_tail()
        for d in range(D):
            self.handler("PUSH%d" % d)
            self.dispatch_head()
            for k in range(K):
                self.e("v_mov_b32_e32 v%d, v%d" % (self.R(d, k), self.T(k)))
            self.dispatch_tail()
        for d in range(D):
            self.handler("PUSHC%d" % d)
            self.dispatch_head(2)
            for k in range(K):
                self.e("v_mov_b32_e32 v%d, v%d" % (self.R(d, k), self.T(k)))
            for k in range(K):
                self.e("v_mov_b32_e32 v%d, %s" % (self.T(k), CA))
            self.dispatch_tail()
        for d in range(D):
            for v in range(NV):
                self.handler("PUSHV%d_%d" % (d, v))
                for k in range(K):
                    self.e("v_mov_b32_e32 v%d, v%d"
                           % (self.R(d, k), self.T(k)))
                self.ldx(self.T(0), v)
                self.dispatch_head()
                self.e("s_waitcnt lgkmcnt(0)")
                self.dispatch_tail()
        for fam in FAMS:
            for d in range(D):
                self.handler("%s_S%d" % (fam, d))
                self.dispatch_head()
                self.binops(fam, ["v%d" % self.R(d, k) for k in range(K)])
                self.dispatch_tail()
            shared = fam in ("div", "rdiv", "ndiv", "nrdiv")
            for v in range(NV):
                self.handler("%s_V%d" % (fam, v))
                self.ldx(self.O(0), v)
                self.dispatch_head()
                if shared:
                    self.e("s_branch .Lbody_%s_V_%%=" % fam)
                    continue
                self.e("s_waitcnt lgkmcnt(0)")
                self.binops(fam, ["v%d" % self.O(k) for k in range(K)])
                self.dispatch_tail()
            if shared:
                self.label(".Lbody_%s_V_" % fam)
                self.e("s_waitcnt lgkmcnt(0)")
                self.binops(fam, ["v%d" % self.O(k) for k in range(K)])
                self.dispatch_tail()
            self.handler("%s_C" % fam)
            self.dispatch_head(2)
            self.binops(fam, [CA] * K)
            self.dispatch_tail()
        self.handler("NEG")
        self.dispatch_head()
        for k in range(K):
            self.e("v_xor_b32_e32 v%d, 0x80000000, v%d"
                   % (self.T(k), self.T(k)))
        self.dispatch_tail()
        for want in ("sin", "cos"):
            self.handler(want.upper())
            self.dispatch_head()
            if self.prio:
                self.e("s_setprio %d" % self.prio[1])
            self.sincos(want)
            if self.prio:
                self.e("s_setprio %d" % self.prio[0])
            self.dispatch_tail()
        self.label(".Lprobe_")
        self.probe_stores(self.POOL0, self.POOL0 + 1)
        self.label(".Lend_")
        if self.prio:
            self.e("s_setprio 0")
        for k in range(K):
            self.e("v_mov_b32_e32 %%[T%d], v%d" % (k, self.T(k)))
        for k in range(K):
            self.e("v_mov_b32_e32 %%[vred%d], v%d" % (k, self.VRED + k))
        self.e("s_mov_b32 m0, s%d" % self.SM0)
        return self


def emit(K, D, NV, suffix="", out_dir=HERE):
    """Writes ``gp_asm_core32<suffix>.inc`` (macros ``GP_ASM_CORE32<SUFFIX>``
    ..., namespace ``asmcore32<suffix>``): the D = 5 core and the deep one."""
    g = Gen32(K, D, NV).build()
    S = suffix.upper()
    lay = g.layout()
    inc = os.path.join(out_dir, "gp_asm_core32%s.inc" % suffix)
    with open(inc, "w") as fh:
        fh.write("// GENERATED by gen_asm32.py (K=%d, D=%d, NV=%d) — do not "
                 "edit\n" % (K, D, NV))
        fh.write("#define GP_ASM_CORE32%s \\\n" % S)
        for l in g.lines:
            fh.write('  "%s\\n" \\\n' % l)
        fh.write('  ""\n')
        clob = ['"v%d"' % r for r in range(g.TB0, g.vmax)]
        clob += ['"s%d"' % r for r in range(g.SB, g.SMAX + 1)]
        clob += ['"vcc"', '"scc"', '"memory"']
        fh.write("#define GP_ASM_CLOBBERS32%s %s\n" % (S, ", ".join(clob)))
        fh.write("#define GP_ASM_T_OUTPUTS32%s %s\n" % (S, ", ".join(
            ['[T%d] "=v"(T[%d])' % (k, k) for k in range(K)] +
            ['[vred%d] "=v"(vred[%d])' % (k, k) for k in range(K)])))
        fh.write("namespace asmcore32%s {\n" % suffix)
        fh.write("constexpr int K = %d, D = %d, NV = %d;\n" % (K, D, NV))
        fh.write("constexpr int VGPRS = %d;\n" % g.vmax)
        for k, v in lay.items():
            if k != "LIM_HI":
                fh.write("constexpr int %s = %d;\n" % (k, v))
        fh.write("constexpr uint32_t LIM = 0x%08x;  // bits of 2^30\n" % LIM32)
        fh.write("constexpr uint32_t INF = 0x%08x;  // bits of +inf\n" % INF32)
        fh.write("// VRED_k = min over sin/cos arguments of 2|x|.bits - 2 LIM:\n"
                 "// < RED_INF re-run, == RED_INF ValueError (gen_asm32.py)\n")
        fh.write("constexpr uint32_t RED_INF = 0x%08x;\n" % RED_INF)
        fh.write("constexpr float kConst[16] = {\n    %s};\n" % ",\n    ".join(
            ["%sf" % float(f32(v)).hex() for _, v in CONSTS] +
            ["0.0f"] * (16 - len(CONSTS))))
        fh.write("}  // namespace asmcore32%s\n" % suffix)
    return inc, lay, g.vmax


if __name__ == "__main__":
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    D = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    NV = int(sys.argv[3]) if len(sys.argv) > 3 else 32
    SUF = sys.argv[4] if len(sys.argv) > 4 else ""
    print(emit(K, D, NV, SUF))
