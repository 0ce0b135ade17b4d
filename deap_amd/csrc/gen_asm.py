#!/usr/bin/env python3
"""Generate the hand-scheduled gfx950 interpreter core (``gp_asm_core.inc``).

The core is one inline-asm block executed by each wavefront of
``f_eval_asm`` (gpeval.hip) for one program over its K cases per lane.  It is
*threaded code*: every program word is the byte offset of a handler relative
to a base label, and every handler ends by fetching the next word with a
scalar load and jumping to it with ``s_setpc_b64`` — no central dispatch
loop, no switch tree, ~6 SALU instructions per node.  Handlers are
specialised by operand-stack slot and by variable index, so the stack lives
in fixed VGPRs (no register indexing, no copies) and variable operands are
read from the LDS case tile with immediate offsets.

Register contract (explicitly numbered, listed as clobbers of the asm):
    v[40 : 40+2K)         T  accumulator, K doubles
    v[RB : RB+2KD)        R  operand stack, slot d case k at RB + 2(dK + k)
    v[OB : OB+2K)         O  operand scratch
    v[TB : TB+2*NT)       sin/cos and division temporaries
    v[VB]                 ValueError bits (bit k: sin/cos saw +-inf)
    s[64:65] handler base, s[66:67] program counter, s[68:69] jump target,
    s70 next word, s71 scratch, s[72:73] inline constant, s74 "redo" flag,
    s75 = 0x3ff00000 (hi word of 1.0), s[76:91] sin/cos constant block,
    s[92:95] lane masks / dummy, s[96:97] constant table, s98 = 0x204.
    Inputs: %[pc] program, %[cst] kTrigConst, %[xa] LDS case tile address,
    %[tab] LDS byte offset of the 64 x (sin hi, lo, cos hi, lo) table.

The same source of truth also emits ``gp_asm_layout.h`` with the handler id
layout the host translator uses (program words -> handler offsets).
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))

FAMS = ["add", "sub", "rsub", "mul", "div", "rdiv"]


class Gen(object):
    def __init__(self, K, D, NV):
        self.K, self.D, self.NV = K, D, NV
        self.TB0 = 40
        self.RB = self.TB0 + 2 * K
        self.OB = self.RB + 2 * K * D
        self.TMP = self.OB + 2 * K
        self.NTMP = 20                      # temp doubles
        self.VB = self.TMP + 2 * self.NTMP
        self.VONE = self.VB + 1             # 0x3ff00000 (hi word of 1.0)
        self.lines = []
        self.handlers = []                  # (name, label)

    # ------------------------------------------------------------ regs --
    @staticmethod
    def p(n):
        return "v[%d:%d]" % (n, n + 1)

    def T(self, k):
        return self.TB0 + 2 * k

    def R(self, d, k):
        return self.RB + 2 * (d * self.K + k)

    def O(self, k):
        return self.OB + 2 * k

    def t(self, i):
        assert i < self.NTMP
        return self.TMP + 2 * i

    def e(self, s):
        self.lines.append(s)

    def label(self, name):
        self.e("%s%%=:" % name)

    # --------------------------------------------------------- dispatch --
    def fetch_next(self, off=0):
        self.e("s_load_dword s70, s[66:67], 0x%x" % off)

    def fetch_const(self):
        self.e("s_load_dword s72, s[66:67], 0x0")
        self.e("s_load_dword s73, s[66:67], 0x4")
        self.fetch_next(8)

    def jump(self, advance):
        self.e("s_add_u32 s66, s66, %d" % advance)
        self.e("s_addc_u32 s67, s67, 0")
        self.e("s_waitcnt lgkmcnt(0)")
        self.e("s_add_u32 s68, s64, s70")
        self.e("s_addc_u32 s69, s65, 0")
        self.e("s_setpc_b64 s[68:69]")

    def handler(self, name):
        lab = ".Lh_%s_" % name
        self.handlers.append((name, lab))
        self.label(lab)

    # ------------------------------------------------------- arithmetic --
    def ldx(self, dst_base, v):
        for k in range(self.K):
            self.e("ds_read_b64 %s, %%[xa] offset:%d"
                   % (self.p(dst_base + 2 * k), (v * self.K + k) * 512))

    def division(self, q, num, den):
        """q = num / den (IEEE, the compiler's gfx950 sequence).
        num/den are operand strings (VGPR pairs)."""
        a, b, c, dd = self.t(16), self.t(17), self.t(18), self.t(19)
        P = self.p
        self.e("v_div_scale_f64 %s, s[92:93], %s, %s, %s" % (P(a), den, den,
                                                             num))
        self.e("v_rcp_f64_e32 %s, %s" % (P(b), P(a)))
        self.e("v_div_scale_f64 %s, vcc, %s, %s, %s" % (P(c), num, den, num))
        self.e("v_fma_f64 %s, -%s, %s, 1.0" % (P(dd), P(a), P(b)))
        self.e("v_fmac_f64_e32 %s, %s, %s" % (P(b), P(b), P(dd)))
        self.e("v_fma_f64 %s, -%s, %s, 1.0" % (P(dd), P(a), P(b)))
        self.e("v_fmac_f64_e32 %s, %s, %s" % (P(b), P(b), P(dd)))
        self.e("v_mul_f64 %s, %s, %s" % (P(dd), P(c), P(b)))
        self.e("v_fma_f64 %s, -%s, %s, %s" % (P(a), P(a), P(dd), P(c)))
        self.e("v_div_fmas_f64 %s, %s, %s, %s" % (P(a), P(a), P(b), P(dd)))
        self.e("v_div_fixup_f64 %s, %s, %s, %s" % (P(q), P(a), den, num))

    def pdiv(self, k, num, den):
        """T_k = (den == 0) ? 1.0 : num / den   (protectedDiv)."""
        q = self.t(15)
        self.division(q, num, den)
        tk = self.T(k)
        self.e("v_cmp_eq_f64_e64 s[94:95], 0, %s" % den)
        self.e("v_cndmask_b32_e64 v%d, v%d, 0, s[94:95]" % (tk, q))
        self.e("v_cndmask_b32_e64 v%d, v%d, v%d, s[94:95]"
               % (tk + 1, q + 1, self.VONE))

    def binop(self, fam, k, a):
        """T_k = fam(a, T_k); a is an operand string (VGPR or SGPR pair)."""
        T = self.p(self.T(k))
        if fam == "add":
            self.e("v_add_f64 %s, %s, %s" % (T, a, T))
        elif fam == "sub":
            self.e("v_add_f64 %s, %s, -%s" % (T, a, T))
        elif fam == "rsub":
            self.e("v_add_f64 %s, %s, -%s" % (T, T, a))
        elif fam == "mul":
            self.e("v_mul_f64 %s, %s, %s" % (T, a, T))
        elif fam == "div":                 # protectedDiv(a, T)
            self.pdiv(k, a, T)
        elif fam == "rdiv":                # protectedDiv(T, a)
            self.pdiv(k, T, a)
        else:
            raise KeyError(fam)

    # ----------------------------------------------------------- sincos --
    def cload(self, block):
        self.e("s_load_dwordx16 s[76:91], s[96:97], 0x%x" % (block * 64))
        self.e("s_waitcnt lgkmcnt(0)")

    @staticmethod
    def c(j):
        """SGPR pair of constant j within the loaded block (0..7)."""
        return "s[%d:%d]" % (76 + 2 * j, 77 + 2 * j)

    def sincos(self, k, want):
        """T_k = sin(T_k) or cos(T_k): gp_trig() of gpeval.hip, operation
        for operation (bit-identical to the C++ kernels).  The 64-entry
        table of sin/cos(j*pi/32) double-doubles sits in LDS at %[tab].
        Constants: block A = INV, C1, C2, LIM, TINY, Ps3, Ps2, Ps1;
        block B = Ps0, Pc2, Pc1, Pc0."""
        P, t, c = self.p, self.t, self.c
        x = P(self.T(k))
        v = self.t                       # VGPR index of temp i
        # ValueError bit (+-inf)
        self.e("v_cmp_class_f64_e64 s[92:93], %s, s98" % x)    # s98 = 0x204
        self.e("v_cndmask_b32_e64 v%d, 0, %d, s[92:93]" % (v(19), 1 << k))
        self.e("v_or_b32_e32 v%d, v%d, v%d" % (self.VB, self.VB, v(19)))
        self.cload(0)
        # redo flag: finite |x| >= 2^40 needs the libm fallback
        self.e("v_cmp_ge_f64_e64 s[92:93], |%s|, %s" % (x, c(3)))
        self.e("s_mov_b32 s71, 0x1f8")
        self.e("v_cmp_class_f64_e64 s[94:95], %s, s71" % x)    # finite
        self.e("s_and_b64 s[92:93], s[92:93], s[94:95]")
        self.e("s_cmp_lg_u64 s[92:93], 0")
        self.e("s_cselect_b32 s71, 1, 0")
        self.e("s_or_b32 s74, s74, s71")
        if want == "sin":               # tiny-argument mask, kept to the end
            self.e("v_cmp_lt_f64_e64 s[92:93], |%s|, %s" % (x, c(4)))
        kd, p1h, p1l, tt, p2h, s1, e1, s2, e2 = [P(t(i)) for i in range(9)]
        tmp = P(t(9))
        self.e("v_mul_f64 %s, %s, %s" % (kd, x, c(0)))
        self.e("v_rndne_f64_e32 %s, %s" % (kd, kd))
        self.e("v_mul_f64 %s, %s, %s" % (p1h, kd, c(1)))
        self.e("v_fma_f64 %s, %s, %s, -%s" % (p1l, kd, c(1), p1h))
        self.e("v_add_f64 %s, %s, -%s" % (tt, x, p1h))
        self.e("v_mul_f64 %s, %s, %s" % (p2h, kd, c(2)))
        self.fast_two_sum(tt, "-" + p1l, s1, e1, tmp)
        self.fast_two_sum(s1, "-" + p2h, s2, e2, tmp)
        rest, rh, rl = P(t(1)), P(t(2)), P(t(4))
        self.e("v_add_f64 %s, %s, %s" % (rest, e1, e2))
        self.fast_two_sum(s2, rest, rh, rl, tmp)
        # j = (kd mod 64) (+16 for cos): kd - 64*floor(kd/64), exact
        kq = P(t(3))
        self.e("v_ldexp_f64 %s, %s, -6" % (kq, kd))
        self.e("v_floor_f64_e32 %s, %s" % (kq, kq))
        self.e("v_ldexp_f64 %s, %s, 6" % (kq, kq))
        self.e("v_add_f64 %s, %s, -%s" % (kq, kd, kq))
        j = v(0)                                 # kd no longer needed
        self.e("v_cvt_i32_f64_e32 v%d, %s" % (j, kq))
        if want == "cos":
            self.e("v_add_u32_e32 v%d, 16, v%d" % (j, j))
        self.e("v_and_b32_e32 v%d, 63, v%d" % (j, j))
        self.e("v_lshlrev_b32_e32 v%d, 5, v%d" % (j, j))
        self.e("v_add_u32_e32 v%d, %%[tab], v%d" % (j, j))
        # sah, sal in t5..t6 ; cah, cal in t7..t8 (v quads)
        self.e("ds_read_b128 v[%d:%d], v%d" % (v(5), v(5) + 3, j))
        self.e("ds_read_b128 v[%d:%d], v%d offset:16" % (v(7), v(7) + 3, j))
        sah, sal, cah, cal = P(t(5)), P(t(6)), P(t(7)), P(t(8))
        zh, zl = P(t(9)), P(t(10))
        self.e("v_mul_f64 %s, %s, %s" % (zh, rh, rh))
        self.e("v_fma_f64 %s, %s, %s, -%s" % (zl, rh, rh, zh))
        ps, pc, tail = P(t(11)), P(t(12)), P(t(13))
        self.e("v_mov_b64_e32 %s, %s" % (pc, c(6)))        # 1 SGPR/instr
        self.e("v_fma_f64 %s, %s, %s, %s" % (ps, c(5), zh, pc))
        self.e("v_fma_f64 %s, %s, %s, %s" % (ps, ps, zh, c(7)))
        self.cload(1)
        self.e("v_fma_f64 %s, %s, %s, %s" % (ps, ps, zh, c(0)))
        self.e("v_mov_b64_e32 %s, %s" % (tail, c(2)))
        self.e("v_fma_f64 %s, %s, %s, %s" % (pc, c(1), zh, tail))
        self.e("v_fma_f64 %s, %s, %s, %s" % (pc, pc, zh, c(3)))
        self.e("v_mul_f64 %s, %s, %s" % (tail, rh, zh))
        self.e("v_mul_f64 %s, %s, %s" % (tail, tail, ps))
        self.e("s_waitcnt lgkmcnt(0)")           # table reads
        p1, q1, m, qm, p2 = [P(t(i)) for i in (14, 15, 16, 17, 18)]
        self.e("v_mul_f64 %s, %s, %s" % (p1, cah, rh))
        self.e("v_fma_f64 %s, %s, %s, -%s" % (q1, cah, rh, p1))
        self.e("v_mul_f64 %s, %s, %s" % (m, sah, zh))
        self.e("v_fma_f64 %s, %s, %s, -%s" % (qm, sah, zh, m))
        self.e("v_mul_f64 %s, -0.5, %s" % (p2, m))
        zlo = zl
        self.e("v_mul_f64 %s, 0.5, %s" % (zlo, zl))
        self.e("v_fma_f64 %s, %s, %s, %s" % (zlo, rh, rl, zlo))
        small = q1
        self.e("v_fma_f64 %s, -0.5, %s, %s" % (small, qm, q1))
        self.e("v_fma_f64 %s, %s, %s, %s" % (small, cah, rl, small))
        self.e("v_fma_f64 %s, %s, %s, %s" % (small, cal, rh, small))
        self.e("v_add_f64 %s, %s, %s" % (small, small, sal))
        self.e("v_fma_f64 %s, -%s, %s, %s" % (small, sah, zlo, small))
        self.e("v_mul_f64 %s, %s, %s" % (pc, zh, pc))
        self.e("v_fma_f64 %s, %s, %s, %s" % (small, m, pc, small))
        self.e("v_fma_f64 %s, %s, %s, %s" % (small, cah, tail, small))
        a_, ae, b_, be = P(t(1)), P(t(3)), P(t(4)), P(t(6))
        res = P(t(19))
        self.fast_two_sum(sah, p1, a_, ae, res)
        self.fast_two_sum(a_, p2, b_, be, res)
        self.e("v_add_f64 %s, %s, %s" % (res, ae, be))
        self.e("v_add_f64 %s, %s, %s" % (res, res, small))
        self.e("v_add_f64 %s, %s, %s" % (res, b_, res))
        tk = self.T(k)
        if want == "sin":
            self.e("v_cndmask_b32_e64 v%d, v%d, v%d, s[92:93]"
                   % (tk, v(19), tk))
            self.e("v_cndmask_b32_e64 v%d, v%d, v%d, s[92:93]"
                   % (tk + 1, v(19) + 1, tk + 1))
        else:
            self.e("v_mov_b64_e32 %s, %s" % (x, res))

    def fast_two_sum(self, a, b, s, e, tmp):
        """s + e = a + b exactly when |a| >= |b| (or a == 0)."""
        self.e("v_add_f64 %s, %s, %s" % (s, a, b))
        self.e("v_add_f64 %s, %s, -%s" % (tmp, s, a))
        self.e("v_add_f64 %s, %s, -%s" % (e, b, tmp))

    def two_sum(self, a, b, s, e, tmp):
        P = self.p
        self.e("v_add_f64 %s, %s, %s" % (s, a, b))
        self.e("v_add_f64 %s, %s, -%s" % (P(tmp), s, a))            # bb
        # e = (a - (s - bb)) + (b - bb)
        self.e("v_add_f64 %s, %s, -%s" % (e, s, P(tmp)))
        self.e("v_add_f64 %s, %s, -%s" % (e, a, e))
        self.e("v_add_f64 %s, %s, -%s" % (P(tmp), b, P(tmp)))
        self.e("v_add_f64 %s, %s, %s" % (e, e, P(tmp)))

    # ----------------------------------------------------------- build --
    def build(self):
        K, D, NV = self.K, self.D, self.NV
        P = self.p
        # prologue
        self.e("s_getpc_b64 s[64:65]")
        self.label(".Lbase_")
        self.e("s_mov_b64 s[66:67], %[pc]")
        self.e("s_mov_b64 s[96:97], %[cst]")
        self.e("s_mov_b32 s74, 0")
        self.e("s_mov_b32 s75, 0x3ff00000")
        self.e("s_mov_b32 s98, 0x204")
        self.e("v_mov_b32_e32 v%d, 0" % self.VB)
        self.e("v_mov_b32_e32 v%d, 0x3ff00000" % self.VONE)
        self.e("s_cmp_eq_u32 %[probe], 0")
        self.e("s_cbranch_scc1 .Lrun_%=")
        self.e("s_branch .Lprobe_%=")
        self.label(".Lrun_")
        self.fetch_next(0)
        self.jump(4)
        # ---- handlers
        self.handler("END")
        self.e("s_branch .Lend_%=")

        self.handler("LDC")
        self.fetch_const()
        self.e("s_waitcnt lgkmcnt(0)")
        for k in range(K):
            self.e("v_mov_b64_e32 %s, s[72:73]" % P(self.T(k)))
        self.jump(12)
        for v in range(NV):
            self.handler("LDV%d" % v)
            self.fetch_next()
            self.ldx(self.T(0), v)
            self.jump(4)
        for d in range(D):
            self.handler("PUSH%d" % d)
            self.fetch_next()
            for k in range(K):
                self.e("v_mov_b64_e32 %s, %s" % (P(self.R(d, k)),
                                                P(self.T(k))))
            self.jump(4)
        for d in range(D):
            self.handler("PUSHC%d" % d)
            self.fetch_const()
            for k in range(K):
                self.e("v_mov_b64_e32 %s, %s" % (P(self.R(d, k)),
                                                P(self.T(k))))
            self.e("s_waitcnt lgkmcnt(0)")
            for k in range(K):
                self.e("v_mov_b64_e32 %s, s[72:73]" % P(self.T(k)))
            self.jump(12)
        for d in range(D):
            for v in range(NV):
                self.handler("PUSHV%d_%d" % (d, v))
                self.fetch_next()
                for k in range(K):
                    self.e("v_mov_b64_e32 %s, %s" % (P(self.R(d, k)),
                                                    P(self.T(k))))
                self.ldx(self.T(0), v)
                self.jump(4)
        for fam in FAMS:
            for d in range(D):
                self.handler("%s_S%d" % (fam, d))
                self.fetch_next()
                for k in range(K):
                    self.binop(fam, k, P(self.R(d, k)))
                self.jump(4)
            for v in range(NV):
                self.handler("%s_V%d" % (fam, v))
                self.fetch_next()
                self.ldx(self.O(0), v)
                self.e("s_waitcnt lgkmcnt(0)")
                for k in range(K):
                    self.binop(fam, k, P(self.O(k)))
                self.jump(4)
            self.handler("%s_C" % fam)
            self.fetch_const()
            self.e("s_waitcnt lgkmcnt(0)")
            for k in range(K):
                self.e("v_mov_b64_e32 %s, s[72:73]" % P(self.O(k)))
            for k in range(K):
                self.binop(fam, k, P(self.O(k)))
            self.jump(12)
        self.handler("NEG")
        self.fetch_next()
        for k in range(K):
            self.e("v_mul_f64 %s, -1.0, %s" % (P(self.T(k)), P(self.T(k))))
        self.jump(4)
        for want in ("sin", "cos"):
            self.handler(want.upper())
            for k in range(K):
                self.sincos(k, want)
            self.fetch_next()
            self.jump(4)
        # ---- probe: write the handler offset table
        self.label(".Lprobe_")
        self.e("v_mov_b32_e32 v%d, 0" % self.t(0))
        for i, (name, lab) in enumerate(self.handlers):
            self.e("v_mov_b32_e32 v%d, %s%%= - .Lbase_%%=" % (self.t(1), lab))
            assert 4 * i < 4096
            self.e("global_store_dword v%d, v%d, %%[probe_out] offset:%d"
                   % (self.t(0), self.t(1), 4 * i))
        self.e("s_waitcnt vmcnt(0)")
        self.label(".Lend_")
        # results out (T to C++ operands, redo flag)
        for k in range(K):
            self.e("v_mov_b64_e32 %%[T%d], %s" % (k, P(self.T(k))))
        self.e("v_mov_b32_e32 %%[vbits], v%d" % self.VB)
        self.e("s_mov_b32 %[redo], s74")
        return self

    def layout(self):
        K, D, NV = self.K, self.D, self.NV
        names = [n for n, _ in self.handlers]
        ids = {n: i for i, n in enumerate(names)}
        # sanity: the arithmetic layout the host uses must match
        base_ldv = ids["LDV0"]
        base_push = ids["PUSH0"]
        base_pushc = ids["PUSHC0"]
        base_pushv = ids["PUSHV0_0"]
        base_bin = ids["add_S0"]
        stride = D + NV + 1
        for f, fam in enumerate(FAMS):
            assert ids["%s_S0" % fam] == base_bin + f * stride
            assert ids["%s_V0" % fam] == base_bin + f * stride + D
            assert ids["%s_C" % fam] == base_bin + f * stride + D + NV
        assert ids["PUSHV%d_%d" % (D - 1, NV - 1)] == \
            base_pushv + (D - 1) * NV + NV - 1
        return {"H_END": ids["END"], "H_LDC": ids["LDC"], "H_LDV0": base_ldv,
                "H_PUSH0": base_push, "H_PUSHC0": base_pushc,
                "H_PUSHV0": base_pushv, "H_BIN0": base_bin,
                "H_FAM_STRIDE": stride, "H_NEG": ids["NEG"],
                "H_SIN": ids["SIN"], "H_COS": ids["COS"],
                "H_COUNT": len(names)}


def trig_data():
    """Table + constants of the table-driven sin/cos (trig_table.json)."""
    import json
    with open(os.path.join(HERE, "trig_table.json")) as fh:
        return json.load(fh)


def trig_const_block():
    """16 doubles the asm core loads as two SGPR blocks of 8:
    block A: INV(32/pi), C1, C2, LIM (2^40), TINY (2^-26), Ps3, Ps2, Ps1
    block B: Ps0, Pc2, Pc1, Pc0, 0, 0, 0, 0."""
    d = trig_data()
    ps, pc = d["Ps"], d["Pc"]
    return ([d["INV"], d["C"][0], d["C"][1], "0x1p+40", "0x1p-26", ps[3],
             ps[2], ps[1]]
            + [ps[0], pc[2], pc[1], pc[0], "0x0p+0", "0x0p+0", "0x0p+0",
               "0x0p+0"])


def emit(K, D, NV, out_dir=HERE):
    g = Gen(K, D, NV).build()
    lay = g.layout()
    body = g.lines
    tag = "k%dd%d" % (K, D)
    inc = os.path.join(out_dir, "gp_asm_core_%s.inc" % tag)
    with open(inc, "w") as fh:
        fh.write("// GENERATED by gen_asm.py (K=%d, D=%d, NV=%d) — do not edit\n"
                 % (K, D, NV))
        fh.write("#define GP_ASM_CORE_%s \\\n" % tag.upper())
        for l in body:
            fh.write('  "%s\\n" \\\n' % l)
        fh.write('  ""\n')
        clob = ['"v%d"' % r for r in range(g.TB0, g.VONE + 1)]
        clob += ['"s%d"' % r for r in range(64, 99)]
        clob += ['"vcc"', '"scc"', '"memory"']
        fh.write("#define GP_ASM_CLOBBERS_%s %s\n" % (tag.upper(),
                                                     ", ".join(clob)))
    hdr = os.path.join(out_dir, "gp_asm_layout_%s.h" % tag)
    with open(hdr, "w") as fh:
        fh.write("// GENERATED by gen_asm.py — handler id layout\n")
        fh.write("namespace asm_%s {\n" % tag)
        fh.write("constexpr int K = %d, D = %d, NV = %d;\n" % (K, D, NV))
        for k, v in lay.items():
            fh.write("constexpr int %s = %d;\n" % (k, v))
        fh.write("constexpr double kTrigConst[16] = {\n    %s};\n"
                 % ",\n    ".join(trig_const_block()))
        fh.write("constexpr double kTrigTable[64 * 4] = {\n    %s};\n"
                 % ",\n    ".join(v for row in trig_data()["table"]
                                   for v in row))
        fh.write("}  // namespace asm_%s\n" % tag)
    return inc, hdr, lay


if __name__ == "__main__":
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    D = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    NV = int(sys.argv[3]) if len(sys.argv) > 3 else 16
    print(emit(K, D, NV))
