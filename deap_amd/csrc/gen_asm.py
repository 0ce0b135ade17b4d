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
    s[92:95] lane masks / dummy, s[96:97] constant table, s98 scratch.

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
        """T_k = sin(T_k) or cos(T_k): gp_sincos() of gpeval.hip, operation
        for operation (bit-identical to the C++ kernels)."""
        P, t, c = self.p, self.t, self.c
        x = P(self.T(k))
        kd, p1h, p1l, tt, p2h, p2l, p3 = [P(t(i)) for i in range(7)]
        s1, e1, s2, e2 = [P(t(i)) for i in range(7, 11)]
        # ValueError bit (+-inf) and redo flag (finite |x| >= 2^20)
        self.e("v_cmp_class_f64_e64 s[92:93], %s, s98" % x)    # s98 = 0x204
        self.e("v_cndmask_b32_e64 v%d, 0, %d, s[92:93]" % (self.t(19), 1 << k))
        self.e("v_or_b32_e32 v%d, v%d, v%d" % (self.VB, self.VB, self.t(19)))
        # block 0: 2/pi, P1, P2, P3, LIM, c3h, c3l, c5h
        self.cload(0)
        self.e("v_cmp_ge_f64_e64 s[92:93], |%s|, %s" % (x, c(4)))
        self.e("s_mov_b32 s71, 0x1f8")
        self.e("v_cmp_class_f64_e64 s[94:95], %s, s71" % x)    # finite
        self.e("s_and_b64 s[92:93], s[92:93], s[94:95]")
        self.e("s_cmp_lg_u64 s[92:93], 0")
        self.e("s_cselect_b32 s71, 1, 0")
        self.e("s_or_b32 s74, s74, s71")
        # reduction
        self.e("v_mul_f64 %s, %s, %s" % (kd, x, c(0)))
        self.e("v_rndne_f64_e32 %s, %s" % (kd, kd))
        self.e("v_mul_f64 %s, %s, %s" % (p1h, kd, c(1)))
        self.e("v_fma_f64 %s, %s, %s, -%s" % (p1l, kd, c(1), p1h))
        self.e("v_add_f64 %s, %s, -%s" % (tt, x, p1h))
        self.e("v_mul_f64 %s, %s, %s" % (p2h, kd, c(2)))
        self.e("v_fma_f64 %s, %s, %s, -%s" % (p2l, kd, c(2), p2h))
        self.e("v_mul_f64 %s, %s, %s" % (p3, kd, c(3)))
        self.two_sum(tt, "-" + p1l, s1, e1, t(11))
        self.two_sum(s1, "-" + p2h, s2, e2, t(11))
        rest, rh, rl = P(t(1)), P(t(2)), P(t(4))      # p1h,p1l,p2h free
        self.e("v_add_f64 %s, %s, %s" % (P(t(12)), e1, e2))
        self.e("v_add_f64 %s, %s, %s" % (P(t(13)), p2l, p3))
        self.e("v_add_f64 %s, %s, -%s" % (rest, P(t(12)), P(t(13))))
        # fast_two_sum(s2, rest) -> rh, rl
        self.e("v_add_f64 %s, %s, %s" % (rh, s2, rest))
        self.e("v_add_f64 %s, %s, -%s" % (P(t(12)), rh, s2))
        self.e("v_add_f64 %s, %s, -%s" % (rl, rest, P(t(12))))
        zh, zl = P(t(5)), P(t(6))
        self.e("v_mul_f64 %s, %s, %s" % (zh, rh, rh))
        self.e("v_fma_f64 %s, %s, %s, -%s" % (zl, rh, rh, zh))
        # keep: kd t0, rh t2, rl t4, zh t5, zl t6; free t1,t3,t7..t18
        # both series are needed: the quadrant picks one of them per lane
        S = self.sin_series(rh, rl, zh, zl)
        C = self.cos_series(rh, rl, zh, zl)
        self.quadrant(k, kd, S, C, want)

    def two_sum(self, a, b, s, e, tmp):
        P = self.p
        self.e("v_add_f64 %s, %s, %s" % (s, a, b))
        self.e("v_add_f64 %s, %s, -%s" % (P(tmp), s, a))            # bb
        # e = (a - (s - bb)) + (b - bb)
        self.e("v_add_f64 %s, %s, -%s" % (e, s, P(tmp)))
        self.e("v_add_f64 %s, %s, -%s" % (e, a, e))
        self.e("v_add_f64 %s, %s, -%s" % (P(tmp), b, P(tmp)))
        self.e("v_add_f64 %s, %s, %s" % (e, e, P(tmp)))

    def sin_series(self, rh, rl, zh, zl):
        """Returns the VGPR pair string holding S (uses t7..t18; result in
        t13).  Blocks: 0 (c3h c3l c5h), 1 (c5l sinQ0..6), 2 (sinQ7)."""
        P, t, c = self.p, self.t, self.c
        r3h, r3l, t3h, t3l = P(t(7)), P(t(8)), P(t(9)), P(t(10))
        r5h, r5l, t5h, t5l = P(t(11)), P(t(12)), P(t(14)), P(t(15))
        # block 0 (c3h, c3l, c5h) is still loaded from the reduction
        # r3 = rh * z   (dd_mul(rh, 0, zh, zl))
        self.e("v_mul_f64 %s, %s, %s" % (r3h, rh, zh))
        self.e("v_fma_f64 %s, %s, %s, -%s" % (r3l, rh, zh, r3h))
        self.e("v_mul_f64 %s, %s, %s" % (P(t(16)), rh, zl))
        self.e("v_mul_f64 %s, 0, %s" % (P(t(17)), zh))
        self.e("v_add_f64 %s, %s, %s" % (P(t(16)), P(t(16)), P(t(17))))
        self.e("v_add_f64 %s, %s, %s" % (r3l, r3l, P(t(16))))
        # t3 = r3 * (1/6)
        self.dd_mul_c(r3h, r3l, 5, 6, t3h, t3l)
        # r5 = r3 * z
        self.e("v_mul_f64 %s, %s, %s" % (r5h, r3h, zh))
        self.e("v_fma_f64 %s, %s, %s, -%s" % (r5l, r3h, zh, r5h))
        self.e("v_mul_f64 %s, %s, %s" % (P(t(16)), r3h, zl))
        self.e("v_mul_f64 %s, %s, %s" % (P(t(17)), r3l, zh))
        self.e("v_add_f64 %s, %s, %s" % (P(t(16)), P(t(16)), P(t(17))))
        self.e("v_add_f64 %s, %s, %s" % (r5l, r5l, P(t(16))))
        # t5 = r5 * (1/120): c5h in block 0 slot 7, c5l in block 1 slot 0
        self.e("v_mul_f64 %s, %s, %s" % (t5h, r5h, c(7)))
        self.e("v_fma_f64 %s, %s, %s, -%s" % (t5l, r5h, c(7), t5h))
        self.e("v_mul_f64 %s, %s, %s" % (P(t(17)), r5l, c(7)))
        self.cload(1)
        self.e("v_mul_f64 %s, %s, %s" % (P(t(16)), r5h, c(0)))
        self.e("v_add_f64 %s, %s, %s" % (P(t(16)), P(t(16)), P(t(17))))
        self.e("v_add_f64 %s, %s, %s" % (t5l, t5l, P(t(16))))
        # q = sinQ Horner from the highest coefficient
        q = P(t(16))
        self.cload(2)
        self.e("v_mov_b64_e32 %s, %s" % (q, c(0)))           # sinQ7
        self.cload(1)
        for j in (7, 6, 5, 4, 3, 2, 1):                      # sinQ6..sinQ0
            self.e("v_fma_f64 %s, %s, %s, %s" % (q, q, zh, c(j)))
        # h7 = (r5h * zh) * q
        self.e("v_mul_f64 %s, %s, %s" % (P(t(17)), r5h, zh))
        self.e("v_mul_f64 %s, %s, %s" % (P(t(17)), P(t(17)), q))
        # a, ae = two_sum(rh, -t3h); b, be = two_sum(a, t5h)
        a, ae, b, be = P(t(7)), P(t(8)), P(t(11)), P(t(12))
        self.two_sum(rh, "-" + t3h, a, ae, t(18))
        self.two_sum(a, t5h, b, be, t(18))
        # stail = (ae + be) + ((t5l - t3l) + (h7 + rl * fma(-0.5, zh, 1.0)))
        self.e("v_fma_f64 %s, -0.5, %s, 1.0" % (P(t(18)), zh))
        self.e("v_mul_f64 %s, %s, %s" % (P(t(18)), rl, P(t(18))))
        self.e("v_add_f64 %s, %s, %s" % (P(t(17)), P(t(17)), P(t(18))))
        self.e("v_add_f64 %s, %s, -%s" % (P(t(18)), t5l, t3l))
        self.e("v_add_f64 %s, %s, %s" % (P(t(17)), P(t(18)), P(t(17))))
        self.e("v_add_f64 %s, %s, %s" % (P(t(18)), ae, be))
        self.e("v_add_f64 %s, %s, %s" % (P(t(17)), P(t(18)), P(t(17))))
        S = P(t(13))
        self.e("v_add_f64 %s, %s, %s" % (S, b, P(t(17))))
        return S

    def dd_mul_c(self, xh, xl, jh, jl, h, l):
        """(h, l) = (xh, xl) * constant pair (c(jh), c(jl)) of block 0."""
        P, t, c = self.p, self.t, self.c
        self.e("v_mul_f64 %s, %s, %s" % (h, xh, c(jh)))
        self.e("v_fma_f64 %s, %s, %s, -%s" % (l, xh, c(jh), h))
        self.e("v_mul_f64 %s, %s, %s" % (P(t(16)), xh, c(jl)))
        self.e("v_mul_f64 %s, %s, %s" % (P(t(17)), xl, c(jh)))
        self.e("v_add_f64 %s, %s, %s" % (P(t(16)), P(t(16)), P(t(17))))
        self.e("v_add_f64 %s, %s, %s" % (l, l, P(t(16))))

    def cos_series(self, rh, rl, zh, zl):
        """C in t3 (uses t1, t3, t7..t12, t14..t18; keeps t13 = S)."""
        P, t, c = self.p, self.t, self.c
        zl2 = P(t(1))
        # zl2 = zl + 2*rh*rl
        self.e("v_mul_f64 %s, 2.0, %s" % (zl2, rh))
        self.e("v_mul_f64 %s, %s, %s" % (zl2, zl2, rl))
        self.e("v_add_f64 %s, %s, %s" % (zl2, zl, zl2))
        t2h, t2l = P(t(7)), P(t(8))
        self.e("v_mul_f64 %s, 0.5, %s" % (t2h, zh))
        self.e("v_mul_f64 %s, 0.5, %s" % (t2l, zl2))
        # z2 = (zh, zl2) * (zh, zl2)
        z2h, z2l = P(t(9)), P(t(10))
        self.e("v_mul_f64 %s, %s, %s" % (z2h, zh, zh))
        self.e("v_fma_f64 %s, %s, %s, -%s" % (z2l, zh, zh, z2h))
        self.e("v_mul_f64 %s, %s, %s" % (P(t(16)), zh, zl2))
        self.e("v_mul_f64 %s, %s, %s" % (P(t(17)), zl2, zh))
        self.e("v_add_f64 %s, %s, %s" % (P(t(16)), P(t(16)), P(t(17))))
        self.e("v_add_f64 %s, %s, %s" % (z2l, z2l, P(t(16))))
        # t4 = z2 * (1/24): c4h, c4l in block 2 slots 1, 2
        self.cload(2)
        t4h, t4l = P(t(11)), P(t(12))
        self.e("v_mul_f64 %s, %s, %s" % (t4h, z2h, c(1)))
        self.e("v_fma_f64 %s, %s, %s, -%s" % (t4l, z2h, c(1), t4h))
        self.e("v_mul_f64 %s, %s, %s" % (P(t(16)), z2h, c(2)))
        self.e("v_mul_f64 %s, %s, %s" % (P(t(17)), z2l, c(1)))
        self.e("v_add_f64 %s, %s, %s" % (P(t(16)), P(t(16)), P(t(17))))
        self.e("v_add_f64 %s, %s, %s" % (t4l, t4l, P(t(16))))
        # q2 Horner: cosQ7 (block 3 slot 2) ... cosQ0 (block 2 slot 3)
        q2 = P(t(14))
        self.cload(3)
        self.e("v_mov_b64_e32 %s, %s" % (q2, c(2)))
        self.e("v_fma_f64 %s, %s, %s, %s" % (q2, q2, zh, c(1)))   # Q6
        self.e("v_fma_f64 %s, %s, %s, %s" % (q2, q2, zh, c(0)))   # Q5
        self.cload(2)
        for j in (7, 6, 5, 4, 3):                                # Q4..Q0
            self.e("v_fma_f64 %s, %s, %s, %s" % (q2, q2, zh, c(j)))
        h6 = P(t(15))
        self.e("v_mul_f64 %s, %s, %s" % (h6, z2h, zh))
        self.e("v_mul_f64 %s, %s, %s" % (h6, h6, q2))
        a, ae, b, be = P(t(9)), P(t(10)), P(t(14)), P(t(16))
        self.two_sum("1.0", "-" + t2h, a, ae, t(18))
        self.two_sum(a, t4h, b, be, t(18))
        # ctail = (ae + be) + ((t4l - t2l) + h6)
        self.e("v_add_f64 %s, %s, -%s" % (P(t(17)), t4l, t2l))
        self.e("v_add_f64 %s, %s, %s" % (P(t(17)), P(t(17)), h6))
        self.e("v_add_f64 %s, %s, %s" % (P(t(18)), ae, be))
        self.e("v_add_f64 %s, %s, %s" % (P(t(17)), P(t(18)), P(t(17))))
        C = P(t(3))
        self.e("v_add_f64 %s, %s, %s" % (C, b, P(t(17))))
        return C

    def quadrant(self, k, kd, S, C, want):
        """quad = (int64)kd & 3; sin: q&1 ? C : S, negate if q&2;
        cos: q&1 ? S : C, negate if (q+1)&2; then the tiny-argument
        overrides and the result into T_k."""
        P, t, c = self.p, self.t, self.c
        x = P(self.T(k))
        qi = self.t(17)
        self.e("v_cvt_i32_f64_e32 v%d, %s" % (qi, kd))   # |kd| < 2^20
        self.e("v_and_b32_e32 v%d, 3, v%d" % (qi, qi))
        one, neg = self.t(18), self.t(18) + 1
        if want == "sin":
            first, second = C, S
            self.e("v_and_b32_e32 v%d, 1, v%d" % (one, qi))
            self.e("v_and_b32_e32 v%d, 2, v%d" % (neg, qi))
        else:
            first, second = S, C
            self.e("v_and_b32_e32 v%d, 1, v%d" % (one, qi))
            self.e("v_add_u32_e32 v%d, 1, v%d" % (neg, qi))
            self.e("v_and_b32_e32 v%d, 2, v%d" % (neg, neg))
        fl = int(first[2:first.index(":")])
        sl = int(second[2:second.index(":")])
        fh, sh = fl + 1, sl + 1
        tk = self.T(k)
        rlo, rhi = self.t(19), self.t(19) + 1
        # pick = (q & 1) ? first : second
        self.e("v_cmp_ne_u32_e32 vcc, 0, v%d" % one)
        self.e("v_cndmask_b32_e32 v%d, v%d, v%d, vcc" % (rlo, sl, fl))
        self.e("v_cndmask_b32_e32 v%d, v%d, v%d, vcc" % (rhi, sh, fh))
        # negate (flip sign bit of the high word) when requested
        self.e("v_lshlrev_b32_e32 v%d, 30, v%d" % (neg, neg))  # 2 -> 1<<31
        self.e("v_xor_b32_e32 v%d, v%d, v%d" % (rhi, rhi, neg))
        # tiny arguments: sin -> x (|x| < 2^-26), cos -> 1 (|x| < 2^-27)
        self.cload(3)
        if want == "sin":
            self.e("v_cmp_lt_f64_e64 vcc, |%s|, %s" % (x, c(3)))
            self.e("v_cndmask_b32_e32 v%d, v%d, v%d, vcc" % (tk, rlo, tk))
            self.e("v_cndmask_b32_e32 v%d, v%d, v%d, vcc" % (tk + 1, rhi,
                                                            tk + 1))
        else:
            self.e("v_cmp_lt_f64_e64 vcc, |%s|, %s" % (x, c(4)))
            self.e("v_cndmask_b32_e64 v%d, v%d, 0, vcc" % (tk, rlo))
            self.e("v_cndmask_b32_e64 v%d, v%d, v%d, vcc"
                   % (tk + 1, rhi, self.VONE))

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


def sincos_constants():
    """The 32-double constant table the core loads in 4 blocks of 8 (C hex
    float literals; the same values as gp_sincos() in gpeval.hip)."""
    return [
        # block 0: 2/pi, pi/2 in three parts, 2^20, 1/3! (hi, lo), 1/5! hi
        "0x1.45f306dc9c883p-1", "0x1.921fb54442d18p+0",
        "0x1.1a62633145c07p-54", "-0x1.f1976b7ed8fbcp-110", "0x1p+20",
        "0x1.5555555555555p-3", "0x1.5555555555555p-57",
        "0x1.1111111111111p-7",
        # block 1: 1/5! lo, sin series r^7.. coefficients Q0..Q6
        "0x1.1111111111111p-63", "-0x1.a01a01a01a01ap-13",
        "0x1.71de3a556c734p-19", "-0x1.ae64567f544e4p-26",
        "0x1.6124613a86d09p-33", "-0x1.ae7f3e733b81fp-41",
        "0x1.952c77030ad4ap-49", "-0x1.2f49b46814157p-57",
        # block 2: sin Q7, 1/4! (hi, lo), cos series r^6.. Q0..Q4
        "0x1.71b8ef6dcf572p-66", "0x1.5555555555555p-5",
        "0x1.5555555555555p-59", "-0x1.6c16c16c16c17p-10",
        "0x1.a01a01a01a01ap-16", "-0x1.27e4fb7789f5cp-22",
        "0x1.1eed8eff8d898p-29", "-0x1.93974a8c07c9dp-37",
        # block 3: cos Q5..Q7, tiny-argument thresholds
        "0x1.ae7f3e733b81fp-45", "-0x1.6827863b97d97p-53",
        "0x1.e542ba4020225p-62", "0x1p-26", "0x1p-27", "0x0p+0", "0x0p+0",
        "0x0p+0"]


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
        fh.write("constexpr double kSinCosConst[32] = {\n    %s};\n"
                 % ",\n    ".join(sincos_constants()))
        fh.write("}  // namespace asm_%s\n" % tag)
    return inc, hdr, lay


if __name__ == "__main__":
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    D = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    NV = int(sys.argv[3]) if len(sys.argv) > 3 else 16
    print(emit(K, D, NV))
