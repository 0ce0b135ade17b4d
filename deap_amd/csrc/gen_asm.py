#!/usr/bin/env python3
"""Generate the hand-scheduled gfx950 interpreter core (``gp_asm_core.inc``).

The core is one inline-asm block executed by each wavefront of
``f_eval_asm`` (gpeval.hip) for one program over its K cases per lane.

Dispatch: *threaded code with an SGPR window*.  Every program word is the
byte offset of a handler relative to a base label.  The program is laid out
by the host in 16-word windows; a window is loaded into 16 SGPRs with one
``s_load_dwordx16`` and M0 indexes the next word inside it, so dispatching a
node is ``s_movrels_b32`` + 64-bit add + ``s_setpc_b64`` — no memory latency
per node.  The host translator ends a window with a RELOAD word that loads
the next one.  Inline constants (two words) are read from the window the
same way.  The dispatch SALU is issued at the top of each handler so it
overlaps the handler's VALU work; ``s_setpc_b64`` ends the handler.

Handlers are specialised by operand-stack slot and by variable index, so the
stack lives in fixed VGPRs (no register indexing, no copies) and variable
operands are read from the LDS case tile with immediate offsets.

sin/cos (``gp_trig`` in gpeval.hip, operation for operation): the K cases of
a lane are independent dependency chains, so the handler interleaves them
instruction by instruction and a linear-scan allocator assigns their
temporaries.  ``k = rint(x*256/pi)`` and ``j = k mod 512`` come from one
magic-constant fma (``x*INV + 1.5*2^52``: the low word is ``k`` in two's
complement); the table holds sin(j pi/256) as double-doubles, so sin reads
entries j and j + 128 and cos entries j + 128 and j + 256 (two
``ds_read_b128``).  Below 2^14 the reduction is one exact fma and one
product (21 fp64 operations per sin/cos); a wave with any argument at or
past 2^14 (or sin's -0.0) runs the mixed body, which also
computes the long reduction and selects per lane as ``gp_trig`` does.
Arguments with ``|x| >= 2^40`` (and inf/nan) are not reduced here: the mixed
body keeps the running max of ``|x|``'s high word in VRED (the fast body's
arguments are below every redo threshold) and the evaluator re-runs such
programs whole with the reference's own sin/cos (``glibc_trig``;
ValueError for inf).

Register contract (explicitly numbered; clobbers of the asm statement):
    v[TB0 : TB0+2K)      T  accumulator, K doubles
    v[RB : RB+2KD)       R  operand stack, slot d case k at RB + 2(dK + k)
    VRED                 max |x|.hi of sin/cos arguments (mixed body)
    temporaries          allocated by the generator; the division temps
                         and O (operand scratch, 2K) live in the same pool
    s[SB : SB+16)        program window (16 words)
    s[SB+16 : SB+32)     trig constants INV, S1, 2^14, -S2, Ps0, Ps1, Pc1, C1
    s[SB+32 : SB+34)     handler base         s[SB+34 : SB+36) window address
    s[SB+36 : SB+38)     jump target          s[SB+38 : SB+40) inline constant
    s[SB+40]             next word            s[SB+41] saved M0
    Inputs: %[pc] first window, %[cst] constant table, %[xa] LDS case tile
    address; VGPR-pair operands the compiler keeps loaded across calls:
    %[mg] = 1.5*2^52, %[ps2] / %[pc2] (the polynomials' last coefficients:
    the constant bus allows one SGPR operand per instruction), and %[one]
    (1.0's high word, protectedDiv).  LDS from byte 0: the 768 x
    (sin hi, lo) table, then (Ps2, Pc2) and (C2, C3) (the mixed body reads
    C2, C3).

The same source of truth also emits ``gp_asm_layout.h`` with the handler id
layout the host translator uses (program words -> handler offsets).
"""
import os
import re
import sys

HERE = os.path.dirname(os.path.abspath(__file__))

FAMS = ["add", "sub", "rsub", "mul", "div", "rdiv", "ndiv", "nrdiv"]
# The typed core (suffix "_typed", PrimitiveSetTyped programs with
# comparisons, logic and if_then_else, counted as hits: spambase.py): the
# flattener's families 0..10 in opcode order (OP_ADD + 3 * fam)
FAMS_TYPED = ["add", "sub", "rsub", "mul", "div", "rdiv", "lt", "gt", "eq",
              "and", "or"]
WINDOW = 16                        # words per SGPR window
MAGIC = "0x1.8p+52"                # 1.5 * 2^52: rint + low-word integer
TINY_HI = 0x3e500000               # high word of 2^-26
LIM_HI = 0x42700000                # high word of 2^40 (beyond: C++ re-run)
# the fast (one-fma) reduction's range: |x| < 2^FAST_EXP
FAST_EXP = int(os.environ.get("GEN_ASM_FAST_EXP", "14"))
FAST_HI = (0x3ff + FAST_EXP) << 20   # high word of 2^FAST_EXP
# the trig constants in the core's SGPR block (kAsmConst, 8 pairs)
SGPR_CONSTS = ["INV", "S1", "FAST", "NS2", "Ps0", "Ps1", "Pc1", "C1"]
# LDS: sin(j pi/256) (hi, lo) for j < 768 at a 16-byte stride, then
# (Ps2, Pc2) and (C2, C3)
TAB_ENTRIES = 768
TAB_BYTES = 16 * TAB_ENTRIES
COS_OFF = 16 * 128                 # entry j + 128
# GEN_ASM_SPLIT_TAB=1 (measurement): the table as two arrays — the 768 high
# parts, then the 768 low parts — read with four ds_read_b64 per call and
# case instead of two ds_read_b128 (same bytes; conflicts priced per
# instruction width)
SPLIT_TAB = os.environ.get("GEN_ASM_SPLIT_TAB", "0") == "1"
# The exact core (suffix "_exact", the redo pass of ill-conditioned
# programs): glibc 2.35's sin/cos (gpeval.hip glibc_trig_t) in the handler.
# Attribution: glibc_ops, glibc_ops2, glibc_seq3, glibc_seq4 and branred_ops
# emit, operation for operation, the algorithms of the GNU C Library 2.35's
# sysdeps/ieee754/dbl-64/s_sin.c (__sin, __cos, do_sin, do_cos,
# reduce_sincos, TAYLOR_SIN) and branred.c (__branred), with the tables of
# sincostab.c and branred.h (Copyright (C) 2001-2022 Free Software
# Foundation, Inc.; IBM Accurate Mathematical Library), distributed under the
# GNU Lesser General Public License, version 2.1 or later.
# LDS from byte 0: __sincostab (440 doubles), then __branred's constants
# (GLIBC_BRANRED_CONSTS, 4 doubles), its toverp table (75 doubles) and one
# pad double, then the case tile.
GLIBC_TAB_BYTES = 440 * 8
GLIBC_BRANRED_BYTES = GLIBC_TAB_BYTES
GLIBC_BRANRED_CONSTS = ["SPLIT", "BBIG1", "BMP2", "PAD"]
# then __sincostab in do_cos's order, (cs, ccs, -sn, -ssn) per entry, at
# GLIBC_COSTAB (glibc_ops2: a cos-type lane's (A, Aa, B, Bb) read directly)
GLIBC_COSTAB = GLIBC_TAB_BYTES + 8 * (4 + 75 + 1)
GLIBC_LDS_BYTES = GLIBC_COSTAB + GLIBC_TAB_BYTES
# The other constants live in registers: 16 pairs in two SGPR blocks (the
# first 16 doubles of the exact core's d_cst), the rest VGPR operands (one
# of an fma's two constants, and hp1's halves, which v_cndmask_b32_e32 takes
# as a VGPR): no per-call LDS reads, no quads held across the handler.
GLIBC_SGPR = ["HPINV", "MP1", "MP2", "PP3", "PP4", "BIG", "HP0", "HP1",
              "SN3", "CS4", "CS2", "S4", "S3", "S2", "S1", "C0126"]
GLIBC_VGPR = ["SN5", "CS6", "S5", "HP1_LO", "HP1_HI"]
BRANRED_HI = 0x419921FB            # |x| >= 105414350: __branred (C++ pass)
# the exact cores' sin/cos: glibc_ops2 (GEN_ASM_GLIBC2=0: glibc_ops, the
# round-3 body with per-lane selects for every path)
GLIBC2 = os.environ.get("GEN_ASM_GLIBC2", "1") == "1"
# glibc_seq3: the EXEC-masked exact sin/cos (GEN_ASM_GLIBC3=0: glibc_ops2)
GLIBC3 = GLIBC2 and os.environ.get("GEN_ASM_GLIBC3", "1") == "1"
# glibc_seq3 with reduce_sincos and TAYLOR_SIN interleaved over the two
# chains (union masks, temporaries, masked final writes)
ILP = os.environ.get("GEN_ASM_EXPERIMENT") == "ilp"
# glibc_seq4 (round 6, the default; GEN_ASM_GLIBC4=0: glibc_seq3): the same
# roundings with fewer VALU instructions per call — one compare per range
# threshold, the do_cos lane masks formed by SALU from them, n holding only
# the negation (bit 31), the result written in place — and __sincostab split
# into three 16-byte-stride arrays (sn, ssn) | (cs, ccs) | (-sn, -ssn), each
# GLIBC_SPLIT_S bytes apart: a ds_read_b128 lane group then spreads over all
# 16 slots of the 256-byte bank row (the 32-byte entries of the interleaved
# table reach only the even slots)
GLIBC4 = GLIBC3 and not ILP and os.environ.get("GEN_ASM_GLIBC4", "1") == "1"
GLIBC_SPLIT_S = 7 * 256            # >= 110 entries x 16 B, a bank-row multiple
GLIBC_T0855 = 0x3feb6000           # |x|.hi < this: |x| < 0.855469 (s_sin.c)
# glibc_seq4's rare blocks (reduce_sincos, the __branred slow path) out of
# line, after the handler's jump (GEN_ASM_OOL=0: in line, branched over)
OOL = os.environ.get("GEN_ASM_OOL", "1") == "1"
# glibc_seq4 with a tiered_late priority: where sin/cos drop to their low
# priority — "wait" (default: once their table gathers have landed),
# "issue" (as soon as the gathers are issued), "join" (after the range blocks)
TRIG_DROP = os.environ.get("GEN_ASM_TRIG_DROP", "wait")
EARLY = os.environ.get("GEN_ASM_EARLY", "1") == "1"
# glibc_seq4 (with EARLY), fewer SALU on the common path: the handler's EXEC
# saved once at the core's entry (no handler leaves EXEC changed), chain 0's
# EXEC restore left to chain 1's first mask op, and the reduce_sincos test a
# branch on the SCC of its mask (EXEC set in the out-of-line block)
SALU = os.environ.get("GEN_ASM_SALU", "1") == "1"
if GLIBC4:
    # LDS from byte 0: the three arrays, __branred's constants, toverp, pad
    GLIBC_BRANRED_BYTES = 3 * GLIBC_SPLIT_S
    GLIBC_COSTAB = None
    GLIBC_LDS_BYTES = GLIBC_BRANRED_BYTES + 8 * (4 + 75 + 1)


class Gen(object):
    def __init__(self, K, D, NV, TB0=32, SB=None, exact=False, trig_group=0,
                 loop=False, typed=False):
        if SB is None:                      # the exact core: 16 more SGPRs
            SB = 40 if exact else 56
        self.K, self.D, self.NV = K, D, NV
        self.exact = exact
        # loop: the core runs the wave's programs one after the other and
        # folds each one's squared errors into its LDS accumulator itself
        # (the lean MSE epilogue); it returns to the caller only at the end
        # of the wave's programs or at a program the caller must finish
        # (redo, an infinite sin/cos argument, a non-finite sum, a tile that
        # is not lean): the caller's state live across the core is then a
        # few registers instead of its whole program loop
        self.loop = loop
        # typed: no sin/cos (no trig constants or table); the STGP families,
        # NOT and if_then_else; the loop's END counts hits (bool(T) is
        # bool(label)) instead of summing squared errors
        self.typed = typed
        self.fams = FAMS_TYPED if typed else FAMS
        self.trig_group = trig_group or int(os.environ.get("GEN_ASM_TRIG_GROUP", "0"))
        # exact core: a wave whose arguments are all below 2.426265 skips
        # glibc's reduce_sincos (GEN_ASM_RSKIP=0: every wave runs it)
        self.rskip = exact and os.environ.get("GEN_ASM_RSKIP", "1") == "1"
        # the case-tile reads of a variable (and the epilogue's target and
        # accumulator reads) two cases per ds_read2st64_b64 (GEN_ASM_READ2)
        self.read2 = os.environ.get("GEN_ASM_READ2", "0") == "1"
        # wave priority (GEN_ASM_PRIO): the default "tiered_late" runs the
        # light handlers (leaves, pushes, add/sub/mul, neg, END) at priority
        # 2, protectedDiv at 1 and sin/cos at 0 from their table gathers on:
        # a wave about to jump to its next handler (whose fetch latency the
        # other waves hide) issues first, and the long VALU bodies fill the
        # gaps (same-box C4: 529.8 -> 520.0 ms).  Measured
        # alternatives: "tiered" (sin/cos at 0 from their entry), "trig_low"
        # (two levels), "trig_high" (inverted, slower); "none": no s_setprio
        pr = os.environ.get("GEN_ASM_PRIO", "tiered_late")
        # (the exact cores: the looped one, the product's fp64 core)
        self.prio = None if typed or (exact and not loop) else \
            {"trig_low": (1, 0), "trig_high": (0, 1), "tiered": (2, 0, 1),
             "tiered_late": (2, 0, 1), "tiered_late_div0": (2, 0, 0),
             "tiered_late_div2": (2, 0), "tiered_late1": (2, 1, 1)}.get(pr)
        # tiered_late*: a sin/cos body drops its priority only once its table
        # gathers are issued
        self.prio_late = self.prio is not None and pr.startswith("tiered_late")
        # handler entries aligned to 2^align bytes (0: packed)
        self.align = int(os.environ.get("GEN_ASM_ALIGN", "0"))
        # the variables' LDS offsets are ds_read immediates (16 bits)
        assert (NV * K - 1) * 512 < 65536, "NV * K too large for LDS offsets"
        self.TB0 = TB0
        self.RB = TB0 + 2 * K
        self.VRED = self.RB + 2 * K * D
        self.VINF = self.VRED + 1           # bit k: an infinite sin/cos argument
        self.POOL0 = self.VRED + 2          # even: first temporary pair
        assert self.POOL0 % 2 == 0
        # operand scratch: inside the temporary pool, above the division
        # temporaries (binop handlers never run sin/cos)
        self.OB = self.POOL0 + 10
        self.vmax = self.OB + 2 * K         # one past the highest VGPR used
        # SGPRs
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
        # exact core: a lane mask pair; NXT (free once the jump target is
        # formed) holds a constant
        self.SMASK = SB + 42
        self.SCONST = self.NXT
        self.TC2 = SB + 44                  # exact core: the 2nd constant block
        if exact:
            self.SMAX = SB + 61          # (SB + 61: glibc_ops2's costab offset)
        # loop cores: the program index j in a core-owned SGPR (%[jio] is read
        # at entry and written at exit only: the compiler may give an input
        # of equal value — the typed core's constant `done` — the same
        # register as %[jio]'s initial value)
        # (the exact core's SMASK and second constant block take SB + 42 ..
        # SB + 59: its loop registers follow them)
        self.SJ = SB + (60 if exact else 42)
        # loop cores: the program whose first window END prefetched into the
        # window SGPRs (~0: none)
        self.SPF = self.SJ + 1
        if loop:
            self.SMAX = max(self.SMAX, self.SPF)
        assert self.SMAX <= 101
        # loop cores: END loads the next program's first window (GEN_ASM_PF,
        # off: neutral on the MSE cores' longer programs; the typed core,
        # GEN_ASM_PF_TYPED, on: C5's 3.8-node programs wait on their window
        # load every tile, kernel 4.14 -> 3.68 ms)
        self.prefetch = loop and (
            os.environ.get("GEN_ASM_PF_TYPED", "1") == "1" if typed else
            os.environ.get("GEN_ASM_PF", "0") == "1")
        # the exact cores with glibc_seq4: M0 saved in a VGPR lane, and the
        # handlers' range compares issued early into free SGPR pairs
        # (GEN_ASM_EARLY=0: M0 in s81, compares one chain at a time)
        self.m0lane = exact and GLIBC4 and EARLY
        self.salu = self.m0lane and SALU and OOL
        self.lines = []
        # code placed after the current handler's jump (out of line): the
        # rare blocks of a handler, so that its common path falls through
        self.ool = []
        self.handlers = []                  # (name, label)

    # ------------------------------------------------------------ regs --
    @staticmethod
    def p(n):
        return "v[%d:%d]" % (n, n + 1)

    @staticmethod
    def sp(n):
        return "s[%d:%d]" % (n, n + 1)

    def T(self, k):
        return self.TB0 + 2 * k

    def R(self, d, k):
        return self.RB + 2 * (d * self.K + k)

    def O(self, k):
        return self.OB + 2 * k

    def tc(self, name):
        """SGPR pair of a trig constant (kAsmConst order)."""
        i = SGPR_CONSTS.index(name)
        return self.sp(self.TC + 2 * i)

    def e(self, s):
        (self.ool if getattr(self, "_in_ool", False) else self.lines).append(s)

    def flush_ool(self):
        """Emit the out-of-line blocks (after the handler's s_setpc_b64)."""
        self.lines.extend(self.ool)
        self.ool = []

    def label(self, name):
        self.e("%s%%=:" % name)

    def use_v(self, hi):
        self.vmax = max(self.vmax, hi + 1)

    # --------------------------------------------------------- dispatch --
    def dispatch_head(self, nconst=0):
        """Read the inline constant (if any) and the next word from the
        window and advance M0.  A program word is the low half of its
        handler's absolute address (the host adds the kernel's base, probed
        once, to the handler offsets; the high half, the same for every
        handler, is set once in the prologue), so the jump target is the
        word itself: two SALU per node.  Issued first so it overlaps the
        handler's VALU/LDS work."""
        W = self.WIN
        if nconst:
            self.e("s_movrels_b32 s%d, s%d" % (self.CA, W))
            self.e("s_movrels_b32 s%d, s%d" % (self.CA + 1, W + 1))
        self.e("s_movrels_b32 s%d, s%d" % (self.TGT, W + nconst))
        self.e("s_add_u32 m0, m0, %d" % (nconst + 1))

    def prologue_base(self):
        """.Lbase (handler offsets are relative to it) and the jump
        target's high half.  With handler alignment (GEN_ASM_ALIGN) .Lbase
        is the aligned start of the handlers, so that every kernel's copy of
        the core has the same offsets whatever its own address."""
        self.e("s_getpc_b64 %s" % self.sp(self.BASE))
        if self.align:
            self.label(".Lpc_")
            self.e("s_add_u32 s%d, s%d, .Lbase_%%= - .Lpc_%%=" % (self.BASE, self.BASE))
            self.e("s_addc_u32 s%d, s%d, 0" % (self.BASE + 1, self.BASE + 1))
        else:
            self.label(".Lbase_")
        self.e("s_mov_b32 s%d, s%d" % (self.TGT + 1, self.BASE + 1))

    def probe_stores(self, t0, t1):
        """The probe path: the handler offset table, then the absolute
        address of .Lbase (lo, hi) after it — this kernel's own copy of the
        core, which the host adds to the offsets."""
        self.e("v_mov_b32_e32 v%d, 0" % t0)
        n = len(self.handlers)
        base = [0]                        # byte offset held in v[t0]

        def store(off):
            # immediate offsets stop at 4095: move the address on past them
            while off - base[0] >= 4096:
                self.e("v_add_u32_e32 v%d, 0x800, v%d" % (t0, t0))
                base[0] += 2048
            self.e("global_store_dword v%d, v%d, %%[probe_out] offset:%d"
                   % (t0, t1, off - base[0]))
        for i, (name, lab) in enumerate(self.handlers):
            self.e("v_mov_b32_e32 v%d, %s%%= - .Lbase_%%=" % (t1, lab))
            store(4 * i)
        for i in range(2):
            self.e("v_mov_b32_e32 v%d, s%d" % (t1, self.BASE + i))
            store(4 * (n + i))
        self.e("s_waitcnt vmcnt(0)")

    def dispatch_tail(self):
        # S_MOVREL needs one wait state after an SALU write of M0: the next
        # handler's first instruction reads M0, so the jump must not follow
        # the M0 update directly
        if self.lines[-1].startswith("s_add_u32 m0"):
            self.e("s_nop 0")
        self.e("s_setpc_b64 %s" % self.sp(self.TGT))

    def late_prio(self, n0):
        """tiered_late: the trig priority set right after the last table
        gather of the body emitted from line n0 on."""
        if not self.prio_late:
            return
        last = max(i for i in range(n0, len(self.lines))
                   if self.lines[i].lstrip().startswith("ds_read"))
        self.lines.insert(last + 1, "s_setprio %d" % self.prio[1])

    def handler(self, name):
        lab = ".Lh_%s_" % name
        self.handlers.append((name, lab))
        if self.align:                   # handler entry on a fetch boundary
            self.e(".p2align %d" % self.align)
        self.label(lab)

    # ------------------------------------------------------- arithmetic --
    def ldx(self, dst_base, v):
        # experiment "dup_ldx" (values unchanged): every variable read issued
        # twice, the marginal cost of the case-tile reads
        rep = 2 if os.environ.get("GEN_ASM_EXPERIMENT") == "dup_ldx" else 1
        if self.read2:
            # two cases per instruction: their tile rows are 512 bytes apart
            # and their registers adjacent (ds_read2st64_b64 offsets count
            # 512-byte rows, 8 bits each)
            for _ in range(rep):
                for k in range(0, self.K - 1, 2):
                    r = v * self.K + k
                    self.e("ds_read2st64_b64 v[%d:%d], %%[xa] offset0:%d offset1:%d"
                           % (dst_base + 2 * k, dst_base + 2 * k + 3, r, r + 1))
                if self.K % 2:
                    self.e("ds_read_b64 %s, %%[xa] offset:%d"
                           % (self.p(dst_base + 2 * (self.K - 1)),
                              (v * self.K + self.K - 1) * 512))
            return
        for k in list(range(self.K)) * rep:
            self.e("ds_read_b64 %s, %%[xa] offset:%d"
                   % (self.p(dst_base + 2 * k), (v * self.K + k) * 512))

    def division(self, q, num, den, tmp):
        """q = num / den (IEEE, the compiler's gfx950 sequence).
        num/den are operand strings (VGPR or SGPR pairs); tmp = 4 pairs."""
        a, b, c, dd = tmp
        P = self.p
        self.e("v_div_scale_f64 %s, vcc, %s, %s, %s" % (P(a), den, den, num))
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

    def division_pair(self, cases, zero_sel=False):
        """division() for two cases at once, interleaved, so that each
        wave has two independent chains in flight (the one-case sequence
        is a single dependent chain of 11 fp64 ops).  cases = [(q, num,
        den, tmp)] * 2.  Only V_DIV_FMAS reads VCC (set by the second
        V_DIV_SCALE), so case 1's scale writes BASE (free once the prologue
        has set the jump target's high half) and is moved to VCC by the
        SALU after case 0's V_DIV_FMAS: the 4-wait-state rule is about VALU
        writes of VCC only, and case 0's VCC write is 8 instructions back."""
        P = self.p
        S = self.sp(self.BASE)
        (q0, n0, d0, t0), (q1, n1, d1, t1) = cases
        regs = [(t0, n0, d0, q0), (t1, n1, d1, q1)]
        for (a, b, c, dd), num, den, q in regs:
            self.e("v_div_scale_f64 %s, vcc, %s, %s, %s" % (P(a), den, den, num))
        for (a, b, c, dd), num, den, q in regs:
            self.e("v_rcp_f64_e32 %s, %s" % (P(b), P(a)))
        for i, ((a, b, c, dd), num, den, q) in enumerate(regs):
            self.e("v_div_scale_f64 %s, %s, %s, %s, %s"
                   % (P(c), "vcc" if i == 0 else S, num, den, num))
        for _ in range(2):
            for (a, b, c, dd), num, den, q in regs:
                self.e("v_fma_f64 %s, -%s, %s, 1.0" % (P(dd), P(a), P(b)))
            for (a, b, c, dd), num, den, q in regs:
                self.e("v_fmac_f64_e32 %s, %s, %s" % (P(b), P(b), P(dd)))
        for (a, b, c, dd), num, den, q in regs:
            self.e("v_mul_f64 %s, %s, %s" % (P(dd), P(c), P(b)))
        for (a, b, c, dd), num, den, q in regs:
            self.e("v_fma_f64 %s, -%s, %s, %s" % (P(a), P(a), P(dd), P(c)))
        for i, ((a, b, c, dd), num, den, q) in enumerate(regs):
            if i:
                self.e("s_mov_b64 vcc, %s" % S)
            self.e("v_div_fmas_f64 %s, %s, %s, %s" % (P(a), P(a), P(b), P(dd)))
        if zero_sel:
            # protectedDiv with the quotient written straight into T: the
            # zero tests read den before a fixup may overwrite it (den or
            # num can be T itself); then only the high word is selected —
            # for den == +-0 the fixup's quotient is +-inf or the default
            # NaN (num nan: its own NaN, default too: set_cases
            # canonicalises the cases' NaNs), low word 0 as 1.0's
            self.e("v_cmp_eq_f64_e64 vcc, 0, %s" % regs[0][2])
            self.e("v_cmp_eq_f64_e64 %s, 0, %s" % (S, regs[1][2]))
        for (a, b, c, dd), num, den, q in regs:
            self.e("v_div_fixup_f64 %s, %s, %s, %s" % (P(q), P(a), den, num))
        if zero_sel:
            self.e("v_cndmask_b32_e32 v%d, v%d, %%[one], vcc" % (regs[0][3] + 1, regs[0][3] + 1))
            self.e("v_cndmask_b32_e64 v%d, v%d, %%[one], %s"
                   % (regs[1][3] + 1, regs[1][3] + 1, S))

    def div_all(self, fam, operands):
        """fam in div/rdiv/ndiv/nrdiv for every case: T_k = fam(a_k, T_k),
        the cases' divisions interleaved two at a time (division_pair);
        then protectedDiv's zero test or numpy's inf/nan test per case."""
        K = self.K
        sets = [[self.POOL0 + 2 * i for i in range(5)],
                [self.OB + 2 * K + 2 * i for i in range(5)]]
        self.use_v(sets[1][4] + 1)
        # protectedDiv's quotient into T directly, one select per case
        # (GEN_ASM_DIV_DIRECT=0: into a temporary, then both words selected)
        direct = fam in ("div", "rdiv") and \
            os.environ.get("GEN_ASM_DIV_DIRECT", "1") == "1"
        k = 0
        while k < K:
            ks = [k, k + 1] if k + 1 < K else [k]
            cases = []
            for j, kk in enumerate(ks):
                T = self.p(self.T(kk))
                num, den = ((operands[kk], T) if fam in ("div", "ndiv")
                            else (T, operands[kk]))
                cases.append((sets[j][4], num, den, sets[j][:4]))
            if len(cases) == 2 and direct:
                cases = [(self.T(kk), num, den, tmp)
                         for (q, num, den, tmp), kk in zip(cases, ks)]
                self.division_pair(cases, zero_sel=True)
                k += 2
                continue
            if len(cases) == 2:
                self.division_pair(cases)
            else:
                q, num, den, tmp = cases[0]
                self.division(q, num, den, tmp)
            for (q, num, den, tmp), kk in zip(cases, ks):
                self.div_select(fam, kk, q, den)
            k += len(ks)

    def div_select(self, fam, k, q, den):
        tk = self.T(k)
        if fam in ("div", "rdiv"):
            self.e("v_cmp_neq_f64_e64 vcc, 0, %s" % den)  # nan: keeps q
        else:
            self.e("s_movk_i32 s%d, 0x1f8" % self.NXT)      # finite classes
            self.e("v_cmp_class_f64_e64 vcc, v[%d:%d], s%d" % (q, q + 1, self.NXT))
        self.e("v_cndmask_b32_e32 v%d, 0, v%d, vcc" % (tk, q))
        self.e("v_cndmask_b32_e32 v%d, %%[one], v%d, vcc" % (tk + 1, q + 1))

    def binop_all(self, fam, operands):
        """binop() for every case k with operand string operands[k]."""
        if fam in ("div", "rdiv", "ndiv", "nrdiv") and \
                os.environ.get("GEN_ASM_DIV_PAIR", "1") == "1":
            tier = self.prio is not None and len(self.prio) > 2
            if tier:
                self.e("s_setprio %d" % self.prio[2])
            self.div_all(fam, operands)
            if tier:
                self.e("s_setprio %d" % self.prio[0])
            return
        for k in range(self.K):
            self.binop(fam, k, operands[k])

    def pdiv(self, k, num, den):
        """T_k = (den == 0) ? 1.0 : num / den   (protectedDiv)."""
        base = self.POOL0
        tmp = [base + 2 * i for i in range(4)]
        q = base + 8
        self.use_v(q + 1)
        self.division(q, num, den, tmp)
        tk = self.T(k)
        self.e("v_cmp_neq_f64_e64 vcc, 0, %s" % den)  # nan: keeps q
        self.e("v_cndmask_b32_e32 v%d, 0, v%d, vcc" % (tk, q))
        self.e("v_cndmask_b32_e32 v%d, %%[one], v%d, vcc" % (tk + 1, q + 1))

    def npdiv(self, k, num, den):
        """T_k = num / den, inf or nan -> 1.0 (symbreg_numpy.py:28-36)."""
        base = self.POOL0
        tmp = [base + 2 * i for i in range(4)]
        q = base + 8
        self.use_v(q + 1)
        self.division(q, num, den, tmp)
        tk = self.T(k)
        # NXT is free once the jump target is formed (dispatch_head)
        self.e("s_movk_i32 s%d, 0x1f8" % self.NXT)          # finite classes
        self.e("v_cmp_class_f64_e64 vcc, v[%d:%d], s%d" % (q, q + 1, self.NXT))
        self.e("v_cndmask_b32_e32 v%d, 0, v%d, vcc" % (tk, q))
        self.e("v_cndmask_b32_e32 v%d, %%[one], v%d, vcc" % (tk + 1, q + 1))

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
        elif fam == "ndiv":                # numpy protectedDiv(a, T)
            self.npdiv(k, a, T)
        elif fam == "nrdiv":               # numpy protectedDiv(T, a)
            self.npdiv(k, T, a)
        elif fam in ("lt", "gt", "eq"):    # (a < T), (T < a), (a == T)
            self.e("v_cmp_%s_f64_e32 vcc, %s, %s" % (fam, a, T))
            self.set_bool(k)
        elif fam in ("and", "or"):         # (a != 0) and/or (T != 0)
            S = self.sp(self.BASE)         # free after the prologue
            self.e("v_cmp_neq_f64_e64 %s, 0, %s" % (S, a))
            self.e("v_cmp_neq_f64_e32 vcc, 0, %s" % T)
            self.e("s_%s_b64 vcc, vcc, %s" % (fam, S))
            self.set_bool(k)
        else:
            raise KeyError(fam)

    def set_bool(self, k):
        """T_k = VCC ? 1.0 : 0.0 (the F machine's bools)."""
        tk = self.T(k)
        self.e("v_mov_b32_e32 v%d, 0" % tk)
        self.e("v_cndmask_b32_e64 v%d, 0, %%[one], vcc" % (tk + 1))

    # ----------------------------------------------------------- sincos --
    def trig_ops(self, k, want, mixed=False):
        """gp_trig() for case k as a list of ops on virtual registers.
        Each op is (template, defs, uses); a template may hold several
        instructions (VCC groups).  Virtual names: pairs unless listed in
        ``singles``/``quads``.  'x' is T_k (fixed), 'VRED'/'tab' fixed."""
        c = self.tc
        ops = []

        def op(t, d=(), u=(), once=False):
            ops.append((t, tuple(d), tuple(u), once))

        def two_sum(a, b, s, e_, tag):         # Knuth TwoSum, 6 ops
            op("v_add_f64 {%s}, %s, %s" % (s, a[0], b[0]), [s], a[1] + b[1])
            op("v_add_f64 {bb%s}, {%s}, -%s" % (tag, s, a[0]),
               ["bb" + tag], [s] + a[1])
            op("v_add_f64 {ta%s}, {%s}, -{bb%s}" % (tag, s, tag),
               ["ta" + tag], [s, "bb" + tag])
            op("v_add_f64 {ta%s}, %s, -{ta%s}" % (tag, a[0], tag),
               ["ta" + tag], a[1] + ["ta" + tag])
            op("v_add_f64 {tb%s}, %s, -{bb%s}" % (tag, b[0], tag),
               ["tb" + tag], b[1] + ["bb" + tag])
            op("v_add_f64 {%s}, {ta%s}, {tb%s}" % (e_, tag, tag), [e_],
               ["ta" + tag, "tb" + tag])

        def V(n, neg=False):
            return (("-{%s}" if neg else "{%s}") % n, [n])

        # Ps2/Pc2 and the rounding constant are asm operands (%[ps2],
        # %[pc2], %[mg]); (C2, C3) of the long reduction follow the table
        if mixed:
            op("v_mov_b32_e32 {cadr}, 0", ["cadr"], [], True)
            op("ds_read_b128 {CL}, {cadr} offset:%d" % (TAB_BYTES + 16),
               ["CL"], ["cadr"], True)
        # kb = 1.5*2^52 + k (%[mg] = 1.5*2^52): its low word is k
        op("v_fma_f64 {kb}, {x}, %s, %%[mg]" % c("INV"), ["kb"], ["x"])
        op("v_add_f64 {kd}, {kb}, -%[mg]", ["kd"], ["kb"])
        # byte offset of entry j = k mod 512 (the table sits at LDS 0); sin
        # reads entries j (S) and j + 128 (C), cos (= sin(x + pi/2)) entries
        # j + 128 and j + 256.  (The rounding constant's mantissa counts k
        # whatever its scale, so the shift to 16-byte entries stays an op.)
        if os.environ.get("GEN_ASM_EXPERIMENT") == "j_lane":
            # experiment (wrong values): entry = lane id, no bank conflicts
            op("v_mbcnt_lo_u32_b32 {j}, -1, 0", ["j"], ["kb"])
        else:
            op("v_and_b32_e32 {j}, 0x1ff, {kb_lo}", ["j"], ["kb"])
        if SPLIT_TAB:
            # hi parts at 8 j, lo parts at TAB_BYTES / 2 + 8 j
            op("v_lshlrev_b32_e32 {j}, 3, {j}", ["j"], ["j"])
            o_s = 8 * 128 if want == "cos" else 0
            lo_off = TAB_BYTES // 2
            for q, part, off in (("SQ", "sh", o_s), ("SQ", "sl", lo_off + o_s),
                                 ("CQ", "ch", o_s + 8 * 128),
                                 ("CQ", "cl", lo_off + o_s + 8 * 128)):
                op("ds_read_b64 {%s}, {j}%s" % (part, " offset:%d" % off if off else ""),
                   [q], ["j"])
        else:
            op("v_lshlrev_b32_e32 {j}, 4, {j}", ["j"], ["j"])
            o_s = COS_OFF if want == "cos" else 0
            op("ds_read_b128 {SQ}, {j}%s" % (" offset:%d" % o_s if o_s else ""),
               ["SQ"], ["j"])
            if os.environ.get("GEN_ASM_EXPERIMENT") == "dup_tab":
                # experiment (values unchanged): the table gathers issued
                # twice, the marginal cost of their bank conflicts
                op("ds_read_b128 {SQ}, {j}%s" % (" offset:%d" % o_s if o_s else ""),
                   ["SQ"], ["j"])
            op("ds_read_b128 {CQ}, {j} offset:%d" % (o_s + COS_OFF), ["CQ"],
               ["j"])
        # fast reduction (|x| < 2^14, |k| < 2^21): t = x - k*S1 exactly
        # (S1 = pi/256 rounded; x - k*S1 fits 53 bits), rl = k*(-S2)
        tname, rlname = ("tf", "rlf") if mixed else ("t", "rl")
        op("v_fma_f64 {%s}, -{kd}, %s, {x}" % (tname, c("S1")), [tname],
           ["kd", "x"])
        op("v_mul_f64 {%s}, {kd}, %s" % (rlname, c("NS2")), [rlname],
           ["kd"])
        if mixed:
            # long reduction (2^14 <= |x| < 2^40): error-free k*C1, two
            # TwoSums, k*C3 folded into the low part (gp_trig, same order)
            op("v_mul_f64 {p1}, {kd}, %s" % c("C1"), ["p1"], ["kd"])
            op("v_fma_f64 {p1e}, {kd}, %s, -{p1}" % c("C1"), ["p1e"],
               ["kd", "p1"])
            op("v_add_f64 {u}, {x}, -{p1}", ["u"], ["x", "p1"])
            op("s_waitcnt lgkmcnt(@NOUT@)", [], [], "wait")
            two_sum(V("u"), V("p1e", True), "s", "e1", "A")
            op("v_mul_f64 {p2}, {kd}, {c2}", ["p2"], ["kd", "CL"])
            op("v_fma_f64 {p2e}, {kd}, {c2}, -{p2}", ["p2e"],
               ["kd", "CL", "p2"])
            two_sum(V("s"), V("p2", True), "s2", "e2", "B")
            op("v_add_f64 {rest}, {e1}, {e2}", ["rest"], ["e1", "e2"])
            op("v_add_f64 {rest}, {rest}, -{p2e}", ["rest"], ["rest", "p2e"])
            op("v_fma_f64 {rest}, -{kd}, {c3}, {rest}", ["rest"],
               ["kd", "CL", "rest"])
            two_sum(V("s2"), V("rest"), "tg", "rlg", "C")
            # per lane: the fast result below 2^14 (as gp_trig chooses)
            op("v_and_b32_e32 {ax}, 0x7fffffff, {x_hi}\n"
               "v_cmp_gt_u32_e32 vcc, 0x%x, {ax}\n"
               "v_cndmask_b32_e32 {t_lo}, {tg_lo}, {tf_lo}, vcc\n"
               "v_cndmask_b32_e32 {t_hi}, {tg_hi}, {tf_hi}, vcc\n"
               "v_cndmask_b32_e32 {rl_lo}, {rlg_lo}, {rlf_lo}, vcc\n"
               "v_cndmask_b32_e32 {rl_hi}, {rlg_hi}, {rlf_hi}, vcc"
               % FAST_HI, ["ax", "t", "rl"], ["x", "tf", "rlf", "tg", "rlg"])
        op("v_add_f64 {rr}, {t}, {rl}", ["rr"], ["t", "rl"])
        op("v_mul_f64 {z}, {rr}, {rr}", ["z"], ["rr"])
        if not mixed:
            op("s_waitcnt lgkmcnt(@NOUT@)", [], [], "wait")
        # Ps(z) = Ps0 + Ps1 z + Ps2 z^2, Pc(z) = -1/2 + Pc1 z + Pc2 z^2
        op("v_fma_f64 {ps}, {z}, %%[ps2], %s" % c("Ps1"), ["ps"], ["z"])
        op("v_fma_f64 {ps}, {ps}, {z}, %s" % c("Ps0"), ["ps"], ["ps", "z"])
        op("v_fma_f64 {pc}, {z}, %%[pc2], %s" % c("Pc1"), ["pc"], ["z"])
        op("v_fma_f64 {pc}, {pc}, {z}, -0.5", ["pc"], ["pc", "z"])
        op("s_waitcnt lgkmcnt(0)", [], [], "wait")
        # a = Sh + Ch*t and its exact error ae (Sh - a is exact)
        op("v_fma_f64 {a}, {ch}, {t}, {sh}", ["a"], ["CQ", "t", "SQ"])
        op("v_add_f64 {d}, {sh}, -{a}", ["d"], ["SQ", "a"])
        op("v_fma_f64 {ae}, {ch}, {t}, {d}", ["ae"], ["CQ", "t", "d"])
        op("v_mul_f64 {h}, {rr}, {ps}", ["h"], ["rr", "ps"])
        op("v_mul_f64 {g}, {ch}, {h}", ["g"], ["CQ", "h"])
        op("v_fma_f64 {tls}, {sh}, {pc}, {g}", ["tls"], ["SQ", "pc", "g"])
        op("v_fma_f64 {sm}, {cl}, {t}, {sl}", ["sm"], ["CQ", "t", "SQ"])
        op("v_fma_f64 {sm}, {ch}, {rl}, {sm}", ["sm"], ["CQ", "rl", "sm"])
        op("v_add_f64 {sm}, {sm}, {ae}", ["sm"], ["sm", "ae"])
        op("v_fma_f64 {sm}, {z}, {tls}, {sm}", ["sm"], ["z", "tls", "sm"])
        if want == "cos" or not mixed:
            # (the prefix sent sin waves with any |x| < 2^-26 to the mixed
            # body)
            op("v_add_f64 {x}, {a}, {sm}", [], ["a", "sm"])
        else:
            op("v_add_f64 {res}, {a}, {sm}", ["res"], ["a", "sm"])
            # |x| < 2^-26: sin(x) rounds to x (keeps -0.0)
            op("v_and_b32_e32 {ax2}, 0x7fffffff, {x_hi}\n"
               "v_cmp_gt_u32_e32 vcc, 0x%x, {ax2}\n"
               "v_cndmask_b32_e64 {x_lo}, {res_lo}, {x_lo}, vcc\n"
               "v_cndmask_b32_e64 {x_hi}, {res_hi}, {x_hi}, vcc"
               % TINY_HI, ["ax2"], ["res", "x"])
        return ops

    def glibc_ops(self, k, want):
        """glibc_trig_t() (gpeval.hip: glibc 2.35 __sin/__cos with one
        do_sincos body per lane) for case k, operation for operation, as a
        list of ops like trig_ops.  Lanes with |x| >= 105414350 (__branred)
        or inf/nan are left to the C++ exact pass (VRED)."""
        cos = want == "cos"
        ops = []

        def const(name):
            if name in GLIBC_VGPR:
                return "%%[g_%s]" % name.lower()
            i = GLIBC_SGPR.index(name)
            return self.sp((self.TC if i < 8 else self.TC2) + 2 * (i % 8))

        def op(t, d=(), u=(), once=False):
            # @NAME@: a constant's register operand
            t = re.sub(r"@([A-Z0-9_]+)@", lambda m: const(m.group(1)), t)
            ops.append((t, tuple(d), tuple(u), once))
        op("v_and_b32_e32 {hx}, 0x7fffffff, {x_hi}", ["hx"], ["x"])
        # |x| < 2.426265: y = hp0 - |x| (sin: do_cos(y, hp1); cos:
        # do_sin(y + hp1, (y - (y + hp1)) + hp1))
        op("v_add_f64 {y}, @HP0@, -|{x}|", ["y"], ["x"])
        if cos:
            op("v_add_f64 {ac}, {y}, @HP1@", ["ac"], ["y"])
            op("v_add_f64 {dac}, {y}, -{ac}", ["dac"], ["y", "ac"])
            op("v_add_f64 {dac}, {dac}, @HP1@", ["dac"], ["dac"])
        # reduce_sincos (skipped by a wave whose every argument is below
        # 2.426265, where the selects below take x itself: rskip)
        op("", [], [], "rskip_beg")
        op("v_fma_f64 {t}, {x}, @HPINV@, %[mg]", ["t"], ["x"])
        op("v_add_f64 {xn}, {t}, -%[mg]", ["xn"], ["t"])
        op("v_fma_f64 {yr}, -{xn}, @MP1@, {x}", ["yr"], ["xn", "x"])
        op("v_fma_f64 {yr}, {xn}, -@MP2@, {yr}", ["yr"], ["xn", "yr"])
        op("v_and_b32_e32 {nr}, 3, {t_lo}", ["nr"], ["t"])
        if cos:
            op("v_add_u32_e32 {nr}, 1, {nr}", ["nr"], ["nr"])
        op("v_fma_f64 {t2}, -{xn}, @PP3@, {yr}", ["t2"], ["xn", "yr"])
        op("v_add_f64 {d1}, {yr}, -{t2}", ["d1"], ["yr", "t2"])
        op("v_fma_f64 {db}, -{xn}, @PP3@, {d1}", ["db"], ["xn", "d1"])
        op("v_fma_f64 {b}, -{xn}, @PP4@, {t2}", ["b"], ["xn", "t2"])
        op("v_add_f64 {d2}, {t2}, -{b}", ["d2"], ["t2", "b"])
        op("v_fma_f64 {dar}, -{xn}, @PP4@, {d2}", ["dar"], ["xn", "d2"])
        op("v_add_f64 {dar}, {dar}, {db}", ["dar"], ["dar", "db"])
        op("", [], [], "rskip_end")
        # (a, da, n): x, 0, cos | reduced | the |x| < 2.426265 transform
        op("v_subrev_u32_e32 {tm}, 0x400368fd, {hx}\n"
           "v_cmp_gt_u32_e32 vcc, 0x%x, {tm}\n"
           "v_cndmask_b32_e32 {a_lo}, {x_lo}, {b_lo}, vcc\n"
           "v_cndmask_b32_e32 {a_hi}, {x_hi}, {b_hi}, vcc\n"
           "v_cndmask_b32_e64 {da_lo}, 0, {dar_lo}, vcc\n"
           "v_cndmask_b32_e64 {da_hi}, 0, {dar_hi}, vcc\n"
           "v_cndmask_b32_e64 {n}, %d, {nr}, vcc"
           % (BRANRED_HI - 0x400368fd, 1 if cos else 0),
           ["tm", "a", "da", "n"], ["hx", "x", "b", "dar", "nr"])
        if cos:
            op("v_subrev_u32_e32 {tm}, 0x3feb6000, {hx}\n"
               "v_cmp_gt_u32_e32 vcc, 0x%x, {tm}\n"
               "v_cndmask_b32_e32 {a_lo}, {a_lo}, {ac_lo}, vcc\n"
               "v_cndmask_b32_e32 {a_hi}, {a_hi}, {ac_hi}, vcc\n"
               "v_cndmask_b32_e32 {da_lo}, {da_lo}, {dac_lo}, vcc\n"
               "v_cndmask_b32_e32 {da_hi}, {da_hi}, {dac_hi}, vcc\n"
               "v_cndmask_b32_e64 {n}, {n}, 0, vcc" % (0x400368fd - 0x3feb6000),
               ["tm", "a", "da", "n"], ["hx", "a", "da", "n", "ac", "dac"])
        else:
            # n = x < 0 ? 3 : 1 (copysign(do_cos(..), x); do_cos > 0 here)
            op("v_lshrrev_b32_e32 {nm}, 30, {x_hi}\n"
               "v_and_or_b32 {nm}, {nm}, 2, 1\n"
               "v_subrev_u32_e32 {tm}, 0x3feb6000, {hx}\n"
               "v_cmp_gt_u32_e32 vcc, 0x%x, {tm}\n"
               "v_cndmask_b32_e32 {a_lo}, {a_lo}, {y_lo}, vcc\n"
               "v_cndmask_b32_e32 {a_hi}, {a_hi}, {y_hi}, vcc\n"
               "v_cndmask_b32_e32 {da_lo}, {da_lo}, @HP1_LO@, vcc\n"
               "v_cndmask_b32_e32 {da_hi}, {da_hi}, @HP1_HI@, vcc\n"
               "v_cndmask_b32_e32 {n}, {n}, {nm}, vcc" % (0x400368fd - 0x3feb6000),
               ["nm", "tm", "a", "da", "n"], ["x", "hx", "a", "da", "n", "y"])
        # |x| >= 105414350: __branred (branred_ops), one block for the chains
        op("", [], [], "branred")
        # do_sincos(a, da, n): isc = n & 1 (do_cos), also as a lane mask M
        # (an SGPR pair per case, free in sin/cos handlers); dx negated if
        # (isc ? a < 0 : a <= 0)
        assert self.K <= 2
        M = "s[%d:%d]" % ((self.CA, self.CA + 1) if k == 0 else
                          (self.BASE, self.BASE + 1))
        op("v_and_b32_e32 {isc}, 1, {n}\n"
           "v_cmp_ne_u32_e64 %s, 0, {isc}" % M, ["isc"], ["n"])
        op("v_xor_b32_e32 {flip}, 1, {isc}\n"
           "v_cmp_eq_f64_e32 vcc, 0, {a}\n"
           "v_lshrrev_b32_e32 {sg}, 31, {a_hi}\n"
           "v_cndmask_b32_e32 {flip}, {sg}, {flip}, vcc\n"
           "v_lshlrev_b32_e32 {flip}, 31, {flip}\n"
           "v_xor_b32_e32 {dxs_hi}, {da_hi}, {flip}\n"
           "v_mov_b32_e32 {dxs_lo}, {da_lo}",
           ["flip", "sg", "dxs"], ["isc", "a", "da"])
        op("v_add_f64 {u}, |{a}|, @BIG@", ["u"], ["a"])
        op("v_add_f64 {q1}, {u}, -@BIG@", ["q1"], ["u"])
        op("v_add_f64 {xr}, |{a}|, -{q1}", ["xr"], ["a", "q1"])
        op("v_add_f64 {vc}, {xr}, {dxs}", ["vc"], ["xr", "dxs"])
        # v = isc ? xr + dx : xr; s1 = isc ? v : dx; s2 = isc ? 0 : dx
        op("v_cndmask_b32_e64 {v_lo}, {xr_lo}, {vc_lo}, %s\n"
           "v_cndmask_b32_e64 {v_hi}, {xr_hi}, {vc_hi}, %s\n"
           "v_cndmask_b32_e64 {s1_lo}, {dxs_lo}, {vc_lo}, %s\n"
           "v_cndmask_b32_e64 {s1_hi}, {dxs_hi}, {vc_hi}, %s\n"
           "v_cndmask_b32_e64 {s2_lo}, {dxs_lo}, 0, %s\n"
           "v_cndmask_b32_e64 {s2_hi}, {dxs_hi}, 0, %s" % ((M,) * 6),
           ["v", "s1", "s2"], ["xr", "vc", "dxs"])
        op("v_mul_f64 {xx}, {v}, {v}", ["xx"], ["v"])
        op("v_mul_f64 {m}, {v}, {xx}", ["m"], ["v", "xx"])
        op("v_fma_f64 {p}, {xx}, @SN5@, @SN3@", ["p"], ["xx"])
        op("v_fma_f64 {tt}, {m}, {p}, {s1}", ["tt"], ["m", "p", "s1"])
        op("v_add_f64 {st}, {tt}, {xr}", ["st"], ["tt", "xr"])
        op("v_cndmask_b32_e64 {s_lo}, {st_lo}, {tt_lo}, %s\n"
           "v_cndmask_b32_e64 {s_hi}, {st_hi}, {tt_hi}, %s" % (M, M),
           ["s"], ["st", "tt"])
        op("v_fma_f64 {w}, {xx}, @CS6@, @CS4@", ["w"], ["xx"])
        op("v_fma_f64 {w}, {w}, {xx}, @CS2@", ["w"], ["w", "xx"])
        op("v_mul_f64 {w}, {w}, {xx}", ["w"], ["w", "xx"])
        op("v_fma_f64 {c}, {s2}, {xr}, {w}", ["c"], ["s2", "xr", "w"])
        # __sincostab entry lo(u) (table at LDS 0): (sn, ssn) at byte 32 lo(u),
        # (cs, ccs) 16 bytes on.  (A, Aa, B, Bb) = sin: (sn, ssn, cs, ccs);
        # cos: (cs, ccs, -sn, -ssn): the two reads' addresses swap per lane
        op("v_lshlrev_b32_e32 {adr}, 4, {isc}\n"
           "v_lshl_add_u32 {adr}, {u_lo}, 5, {adr}\n"
           "v_xor_b32_e32 {adr2}, 16, {adr}", ["adr", "adr2"], ["isc", "u"])
        op("ds_read_b128 {EA}, {adr}", ["EA"], ["adr"])
        op("ds_read_b128 {EB}, {adr2}", ["EB"], ["adr2"])
        op("s_waitcnt lgkmcnt(0)", [], [], "wait")
        op("v_lshlrev_b32_e32 {sgn}, 31, {isc}\n"
           "v_xor_b32_e32 {TB_hi}, {TB_hi}, {sgn}\n"
           "v_xor_b32_e32 {TBb_hi}, {TBb_hi}, {sgn}", ["sgn", "EB"], ["isc", "EB"])
        op("v_fma_f64 {cor}, {s}, {TBb}, {TAa}", ["cor"], ["s", "EB", "EA"])
        op("v_fma_f64 {cor}, -{c}, {TA}, {cor}", ["cor"], ["c", "EA", "cor"])
        op("v_fma_f64 {cor}, {s}, {TB}, {cor}", ["cor"], ["s", "EB", "cor"])
        op("v_add_f64 {r}, {TA}, {cor}", ["r"], ["EA", "cor"])
        # do_sin: copysign(sn + cor, a)
        op("s_mov_b32 s%d, 0x7fffffff\n"
           "v_bfi_b32 {rc}, s%d, {r_hi}, {a_hi}\n"
           "v_cndmask_b32_e64 {r_hi}, {rc}, {r_hi}, %s"
           % (self.SCONST, self.SCONST, M), ["rc", "r"], ["r", "a"])
        # do_sin with |a| < 0.126: TAYLOR_SIN(a*a, a, da)
        op("v_mul_f64 {xx2}, {a}, {a}", ["xx2"], ["a"])
        op("v_fma_f64 {pt}, {xx2}, @S5@, @S4@", ["pt"], ["xx2"])
        op("v_fma_f64 {pt}, {pt}, {xx2}, @S3@", ["pt"], ["pt", "xx2"])
        op("v_fma_f64 {pt}, {pt}, {xx2}, @S2@", ["pt"], ["pt", "xx2"])
        op("v_fma_f64 {pt}, {pt}, {xx2}, @S1@", ["pt"], ["pt", "xx2"])
        op("v_mul_f64 {h}, {da}, 0.5", ["h"], ["da"])
        op("v_fma_f64 {q}, {pt}, {a}, -{h}", ["q"], ["pt", "a", "h"])
        op("v_fma_f64 {q}, {q}, {xx2}, {da}", ["q"], ["q", "xx2", "da"])
        op("v_add_f64 {q}, {a}, {q}", ["q"], ["a", "q"])
        op("v_cmp_gt_f64_e64 vcc, @C0126@, |{a}|\n"
           "s_andn2_b64 vcc, vcc, %s\n"
           "v_cndmask_b32_e32 {r_lo}, {r_lo}, {q_lo}, vcc\n"
           "v_cndmask_b32_e32 {r_hi}, {r_hi}, {q_hi}, vcc" % M,
           ["r"], ["a", "r", "q"])
        # (n & 2): -r
        op("v_and_b32_e32 {ng}, 2, {n}\n"
           "v_lshlrev_b32_e32 {ng}, 30, {ng}\n"
           "v_xor_b32_e32 {r_hi}, {r_hi}, {ng}", ["ng", "r"], ["n", "r"])
        # tiny |x|: sin(x) = x, cos(x) = 1
        if cos:
            op("v_cmp_gt_u32_e32 vcc, 0x3e400000, {hx}\n"
               "v_cndmask_b32_e64 {x_lo}, {r_lo}, 0, vcc\n"
               "v_cndmask_b32_e32 {x_hi}, {r_hi}, %[one], vcc", [], ["hx", "r"])
        else:
            op("v_cmp_gt_u32_e32 vcc, 0x3e500000, {hx}\n"
               "v_cndmask_b32_e32 {x_lo}, {r_lo}, {x_lo}, vcc\n"
               "v_cndmask_b32_e32 {x_hi}, {r_hi}, {x_hi}, vcc", [], ["hx", "r"])
        return ops

    def glibc_ops2(self, k, want):
        """glibc_trig_t() (gpeval.hip: glibc 2.35 __sin/__cos, one do_sincos
        body per lane) for case k, with every rounding of glibc's own and
        fewer per-lane selects than glibc_ops: wave-uniform skips of the
        pieces no lane needs (the 0.855469 <= |x| < 2.426265 transform,
        reduce_sincos, __branred, TAYLOR_SIN), do_sin and do_cos bodies of
        their own for waves whose lanes are all of one kind (the merged body
        only for mixed waves), the cos-type lanes' table entries read from a
        cos-ordered copy of __sincostab (no sign flips), dx signed by one
        xor (for da != 0, a is never +-0: x is no multiple of pi/2; for
        da == 0 the sign of dx changes no rounding), and one sign fix
        (copysign for do_sin, the n & 2 negation) at the end.  Lanes with
        inf/nan arguments are left to the C++ exact pass (VRED)."""
        assert not GLIBC4, "glibc_ops2 reads the interleaved table layout"
        cos = want == "cos"
        ops = []

        def const(name):
            if name in GLIBC_VGPR:
                return "%%[g_%s]" % name.lower()
            i = GLIBC_SGPR.index(name)
            return self.sp((self.TC if i < 8 else self.TC2) + 2 * (i % 8))

        def op(t, d=(), u=(), once=False):
            t = re.sub(r"@([A-Z0-9_]+)@", lambda m: const(m.group(1)), t)
            ops.append((t, tuple(d), tuple(u), once))
        M = self.sp(self.CA) if k == 0 else self.sp(self.BASE)
        SK = self.sp(self.SMASK)
        W = "%s_%%=" % want

        def skip(test, d, u, label):
            """a block that runs only if `test` (sets VCC) holds for some
            active lane of some chain"""
            op(test, d, u, ("need", SK))
            op("", [], [], ("skipto", SK, label))
        # ---- (a, da, n): x, 0, cos for |x| < 0.855469
        op("v_and_b32_e32 {hx}, 0x7fffffff, {x_hi}\n"
           "v_max_u32_e32 v%d, v%d, {hx}" % (self.VRED, self.VRED), ["hx"], ["x"])
        op("v_mov_b64_e32 {a}, {x}\nv_mov_b64_e32 {da}, 0\n"
           "v_mov_b32_e32 {n}, %d" % (1 if cos else 0), ["a", "da", "n"], ["x"])
        # ---- 0.855469 <= |x| < 2.426265: y = hp0 - |x| (sin: do_cos(y, hp1),
        # sign of x; cos: do_sin(y + hp1, (y - (y + hp1)) + hp1))
        dtest = ("v_subrev_u32_e32 {tm}, 0x3feb6000, {hx}\n"
                 "v_cmp_gt_u32_e32 vcc, 0x%x, {tm}" % (0x400368fd - 0x3feb6000))
        skip(dtest, ["tm"], ["hx"], ".Ld_" + W)
        op("v_add_f64 {y}, @HP0@, -|{x}|", ["y"], ["x"])
        if cos:
            op("v_add_f64 {ac}, {y}, @HP1@", ["ac"], ["y"])
            op("v_add_f64 {dac}, {y}, -{ac}", ["dac"], ["y", "ac"])
            op("v_add_f64 {dac}, {dac}, @HP1@", ["dac"], ["dac"])
            op("v_cmp_gt_u32_e32 vcc, 0x%x, {tm}\n"
               "v_cndmask_b32_e32 {a_lo}, {a_lo}, {ac_lo}, vcc\n"
               "v_cndmask_b32_e32 {a_hi}, {a_hi}, {ac_hi}, vcc\n"
               "v_cndmask_b32_e32 {da_lo}, {da_lo}, {dac_lo}, vcc\n"
               "v_cndmask_b32_e32 {da_hi}, {da_hi}, {dac_hi}, vcc\n"
               "v_cndmask_b32_e64 {n}, {n}, 0, vcc" % (0x400368fd - 0x3feb6000),
               ["a", "da", "n"], ["tm", "a", "da", "n", "ac", "dac"])
        else:
            op("v_lshrrev_b32_e32 {nm}, 30, {x_hi}\n"
               "v_and_or_b32 {nm}, {nm}, 2, 1\n"
               "v_cmp_gt_u32_e32 vcc, 0x%x, {tm}\n"
               "v_cndmask_b32_e32 {a_lo}, {a_lo}, {y_lo}, vcc\n"
               "v_cndmask_b32_e32 {a_hi}, {a_hi}, {y_hi}, vcc\n"
               "v_cndmask_b32_e32 {da_lo}, {da_lo}, @HP1_LO@, vcc\n"
               "v_cndmask_b32_e32 {da_hi}, {da_hi}, @HP1_HI@, vcc\n"
               "v_cndmask_b32_e32 {n}, {n}, {nm}, vcc" % (0x400368fd - 0x3feb6000),
               ["nm", "a", "da", "n"], ["x", "tm", "a", "da", "n", "y"])
        op("", [], [], ("label", ".Ld_" + W))
        # ---- 2.426265 <= |x| < 105414350: reduce_sincos
        skip("v_cmp_le_u32_e32 vcc, 0x400368fd, {hx}", [], ["hx"], ".Le_" + W)
        op("v_fma_f64 {t}, {x}, @HPINV@, %[mg]", ["t"], ["x"])
        op("v_add_f64 {xn}, {t}, -%[mg]", ["xn"], ["t"])
        op("v_fma_f64 {yr}, -{xn}, @MP1@, {x}", ["yr"], ["xn", "x"])
        op("v_fma_f64 {yr}, {xn}, -@MP2@, {yr}", ["yr"], ["xn", "yr"])
        op("v_and_b32_e32 {nr}, 3, {t_lo}", ["nr"], ["t"])
        if cos:
            op("v_add_u32_e32 {nr}, 1, {nr}", ["nr"], ["nr"])
        op("v_fma_f64 {t2}, -{xn}, @PP3@, {yr}", ["t2"], ["xn", "yr"])
        op("v_add_f64 {d1}, {yr}, -{t2}", ["d1"], ["yr", "t2"])
        op("v_fma_f64 {db}, -{xn}, @PP3@, {d1}", ["db"], ["xn", "d1"])
        op("v_fma_f64 {b}, -{xn}, @PP4@, {t2}", ["b"], ["xn", "t2"])
        op("v_add_f64 {d2}, {t2}, -{b}", ["d2"], ["t2", "b"])
        op("v_fma_f64 {dar}, -{xn}, @PP4@, {d2}", ["dar"], ["xn", "d2"])
        op("v_add_f64 {dar}, {dar}, {db}", ["dar"], ["dar", "db"])
        op("v_subrev_u32_e32 {tm}, 0x400368fd, {hx}\n"
           "v_cmp_gt_u32_e32 vcc, 0x%x, {tm}\n"
           "v_cndmask_b32_e32 {a_lo}, {a_lo}, {b_lo}, vcc\n"
           "v_cndmask_b32_e32 {a_hi}, {a_hi}, {b_hi}, vcc\n"
           "v_cndmask_b32_e32 {da_lo}, {da_lo}, {dar_lo}, vcc\n"
           "v_cndmask_b32_e32 {da_hi}, {da_hi}, {dar_hi}, vcc\n"
           "v_cndmask_b32_e32 {n}, {n}, {nr}, vcc" % (BRANRED_HI - 0x400368fd),
           ["tm", "a", "da", "n"], ["hx", "a", "da", "n", "b", "dar", "nr"])
        op("", [], [], ("label", ".Le_" + W))
        # ---- |x| >= 105414350: __branred (branred_ops), one block for the chains
        op("", [], [], "branred")
        # ---- do_sincos(a, da, n): isc = n & 1 (M: this chain's lane mask)
        op("v_and_b32_e32 {isc}, 1, {n}\n"
           "v_cmp_ne_u32_e64 %s, 0, {isc}" % M, ["isc"], ["n"])
        # dx signed as do_sin / do_cos sign it (|a| below)
        op("v_and_b32_e32 {sg}, 0x80000000, {a_hi}\n"
           "v_xor_b32_e32 {dxs_hi}, {da_hi}, {sg}\n"
           "v_mov_b32_e32 {dxs_lo}, {da_lo}", ["sg", "dxs"], ["a", "da"])
        op("v_add_f64 {u}, |{a}|, @BIG@", ["u"], ["a"])
        op("v_add_f64 {q1}, {u}, -@BIG@", ["q1"], ["u"])
        op("v_lshlrev_b32_e32 {adr0}, 5, {u_lo}", ["adr0"], ["u"])
        op("v_add_f64 {xr}, |{a}|, -{q1}", ["xr"], ["a", "q1"])
        # the three bodies: their temporaries named per body (their live
        # ranges stay inside it); r, the result, is shared (one register)
        def body(kind):
            def N(v):
                return v + "_" + kind
            def t(tmpl):                 # {name} -> {name_<kind>}, r and the
                return re.sub(r"\{([a-zA-Z0-9]+)(_lo|_hi)?\}",   # live-ins kept
                              lambda m: "{%s%s}" % (
                                  m.group(1) if m.group(1) in
                                  ("r", "xr", "dxs", "adr0", "a", "isc") else N(m.group(1)),
                                  m.group(2) or ""), tmpl)
            def o(tmpl, d, u, once=False):
                ren = lambda vs: [v if v in ("r", "xr", "dxs", "adr0", "a", "isc") else N(v)
                                  for v in vs]
                op(t(tmpl), ren(d), ren(u), once)
            # (A, Aa, B, Bb) at 32 lo(u): __sincostab, or its cos-ordered copy
            if kind == "m":
                o("v_mad_u32_u24 {adr}, {isc}, s%d, {adr0}" % self.SPF,
                  ["adr"], ["isc", "adr0"])
                tab, A = 0, "adr"
            else:
                tab, A = (GLIBC_COSTAB if kind == "c" else 0), "adr0"
            if kind == "m":
                # v = isc ? xr + dx : xr; s1 = isc ? v : dx; s2 = isc ? 0 : dx
                o("v_add_f64 {vc}, {xr}, {dxs}", ["vc"], ["xr", "dxs"])
                o("v_cndmask_b32_e64 {v_lo}, {xr_lo}, {vc_lo}, %s\n"
                  "v_cndmask_b32_e64 {v_hi}, {xr_hi}, {vc_hi}, %s\n"
                  "v_cndmask_b32_e64 {s1_lo}, {dxs_lo}, {vc_lo}, %s\n"
                  "v_cndmask_b32_e64 {s1_hi}, {dxs_hi}, {vc_hi}, %s" % ((M,) * 4),
                  ["v", "s1"], ["xr", "vc", "dxs"])
                v, s1 = "v", "s1"
            elif kind == "c":
                o("v_add_f64 {v}, {xr}, {dxs}", ["v"], ["xr", "dxs"])
                v = s1 = "v"
            else:
                v, s1 = "xr", "dxs"
            V = "{%s}" % v if v == "xr" else "{%s}" % v
            S1 = "{%s}" % s1
            o("v_mul_f64 {xx}, %s, %s" % (V, V), ["xx"], [v])
            o("v_mul_f64 {m}, %s, {xx}" % V, ["m"], [v, "xx"])
            o("v_fma_f64 {p}, {xx}, @SN5@, @SN3@", ["p"], ["xx"])
            if kind == "c":                 # s = t
                o("v_fma_f64 {s}, {m}, {p}, %s" % S1, ["s"], ["m", "p", s1])
            else:
                o("v_fma_f64 {tt}, {m}, {p}, %s" % S1, ["tt"], ["m", "p", s1])
                if kind == "s":
                    o("v_add_f64 {s}, {tt}, {xr}", ["s"], ["tt", "xr"])
                else:
                    o("v_add_f64 {st}, {tt}, {xr}", ["st"], ["tt", "xr"])
                    o("v_cndmask_b32_e64 {s_lo}, {st_lo}, {tt_lo}, %s\n"
                      "v_cndmask_b32_e64 {s_hi}, {st_hi}, {tt_hi}, %s" % (M, M),
                      ["s"], ["st", "tt"])
            o("v_fma_f64 {w}, {xx}, @CS6@, @CS4@", ["w"], ["xx"])
            o("v_fma_f64 {w}, {w}, {xx}, @CS2@", ["w"], ["w", "xx"])
            o("v_mul_f64 {w}, {w}, {xx}", ["w"], ["w", "xx"])
            o("ds_read_b128 {EA}, {%s} offset:%d" % (A, tab), ["EA"], [A])
            o("ds_read_b128 {EB}, {%s} offset:%d" % (A, tab + 16), ["EB"], [A])
            if kind == "m":                 # c = fma(isc ? 0 : dx, xr, w)
                o("v_cndmask_b32_e64 {s2_lo}, {dxs_lo}, 0, %s\n"
                  "v_cndmask_b32_e64 {s2_hi}, {dxs_hi}, 0, %s" % (M, M),
                  ["s2"], ["dxs"])
                o("v_fma_f64 {c}, {s2}, {xr}, {w}", ["c"], ["s2", "xr", "w"])
                C = "c"
            elif kind == "s":
                o("v_fma_f64 {c}, {dxs}, {xr}, {w}", ["c"], ["dxs", "xr", "w"])
                C = "c"
            else:
                C = "w"                     # do_cos: c = w
            op("s_waitcnt lgkmcnt(0)", [], [], "wait")
            if self.prio:
                op("s_setprio %d" % self.prio[1], [], [], ("once",))
            o("v_fma_f64 {cor}, {s}, {TBb}, {TAa}", ["cor"], ["s", "EB", "EA"])
            o("v_fma_f64 {cor}, -{%s}, {TA}, {cor}" % C, ["cor"], [C, "EA", "cor"])
            o("v_fma_f64 {cor}, {s}, {TB}, {cor}", ["cor"], ["s", "EB", "cor"])
            o("v_add_f64 {r}, {TA}, {cor}", ["r"], ["EA", "cor"])
        # waves of one kind take their own body (k = K - 1 decides for all)
        op("s_or_b64 %s, s[%d:%d], s[%d:%d]\n"
           "s_and_b64 %s, exec, %s\n"
           "s_cbranch_scc0 .Lbs_%s\n"
           "s_and_b64 %s, s[%d:%d], s[%d:%d]\n"
           "s_andn2_b64 %s, exec, %s\n"
           "s_cbranch_scc0 .Lbc_%s"
           % (SK, self.CA, self.CA + 1, self.BASE, self.BASE + 1, SK, SK, W,
              SK, self.CA, self.CA + 1, self.BASE, self.BASE + 1, SK, SK, W),
           [], [], ("once",))
        body("m")                          # lanes of both kinds
        op("s_branch .Lbe_%s" % W, [], [], ("once",))
        op("", [], [], ("label", ".Lbs_" + W))
        body("s")                          # every lane do_sin
        op("s_branch .Lbe_%s" % W, [], [], ("once",))
        op("", [], [], ("label", ".Lbc_" + W))
        body("c")                          # every lane do_cos
        op("", [], [], ("label", ".Lbe_" + W))
        # do_sin's copysign(r, a) (r > 0 here)
        op("v_and_b32_e32 {sa}, 0x80000000, {a_hi}\n"
           "v_cndmask_b32_e64 {sa}, {sa}, 0, %s\n"
           "v_xor_b32_e32 {r_hi}, {r_hi}, {sa}" % M, ["sa", "r"], ["a", "r"])
        # do_sin with |a| < 0.126: TAYLOR_SIN(a*a, a, da) (sin-type lanes)
        ttest = ("v_cmp_gt_f64_e64 vcc, @C0126@, |{a}|\n"
                 "s_andn2_b64 vcc, vcc, %s" % M)
        skip(ttest, [], ["a"], ".Lt_" + W)
        op("v_mul_f64 {xx2}, {a}, {a}", ["xx2"], ["a"])
        op("v_fma_f64 {pt}, {xx2}, @S5@, @S4@", ["pt"], ["xx2"])
        op("v_fma_f64 {pt}, {pt}, {xx2}, @S3@", ["pt"], ["pt", "xx2"])
        op("v_fma_f64 {pt}, {pt}, {xx2}, @S2@", ["pt"], ["pt", "xx2"])
        op("v_fma_f64 {pt}, {pt}, {xx2}, @S1@", ["pt"], ["pt", "xx2"])
        op("v_mul_f64 {h}, {da}, 0.5", ["h"], ["da"])
        op("v_fma_f64 {q}, {pt}, {a}, -{h}", ["q"], ["pt", "a", "h"])
        op("v_fma_f64 {q}, {q}, {xx2}, {da}", ["q"], ["q", "xx2", "da"])
        op("v_add_f64 {q}, {a}, {q}", ["q"], ["a", "q"])
        op(ttest + "\n"
           "v_cndmask_b32_e32 {r_lo}, {r_lo}, {q_lo}, vcc\n"
           "v_cndmask_b32_e32 {r_hi}, {r_hi}, {q_hi}, vcc", ["r"], ["a", "r", "q"])
        op("", [], [], ("label", ".Lt_" + W))
        # (n & 2): -r
        op("v_and_b32_e32 {ng}, 2, {n}\n"
           "v_lshlrev_b32_e32 {ng}, 30, {ng}\n"
           "v_xor_b32_e32 {r_hi}, {r_hi}, {ng}", ["ng", "r"], ["n", "r"])
        # tiny |x|: sin(x) = x, cos(x) = 1
        if cos:
            op("v_cmp_gt_u32_e32 vcc, 0x3e400000, {hx}\n"
               "v_cndmask_b32_e64 {x_lo}, {r_lo}, 0, vcc\n"
               "v_cndmask_b32_e32 {x_hi}, {r_hi}, %[one], vcc", [], ["hx", "r"])
        else:
            op("v_cmp_gt_u32_e32 vcc, 0x3e500000, {hx}\n"
               "v_cndmask_b32_e32 {x_lo}, {r_lo}, {x_lo}, vcc\n"
               "v_cndmask_b32_e32 {x_hi}, {r_hi}, {x_hi}, vcc", [], ["hx", "r"])
        return ops

    def glibc_seq3(self, want):
        """glibc_trig_t() (gpeval.hip: glibc 2.35 __sin/__cos) for the K = 2
        chains as one allocator seq, every rounding of glibc's own as in
        glibc_ops2, but the per-lane choices made with the EXEC mask instead
        of v_cndmask selects (a select of a double is two VALU instructions,
        as many as an fma: round 5's profile showed the select glue at 60 %
        of the exact core's VALU instructions).  Each range block (0.855469 <=
        |x| < 2.426265, reduce_sincos, __branred) is a wave-uniform skip, then
        per chain under its lane mask writes (a, da, n) in place; a is x's own
        register (the blocks read x before they write it, and lanes outside
        every block keep a = x).  do_sin and do_cos share one body: the cos
        lanes fold dx into xr (v) and dx := v before it, the sin lanes add xr
        and x*dx after it; TAYLOR_SIN and sin's tiny |x| run under the do_sin
        lanes' mask; the n & 2 negation is one integer add into the result's
        sign bit.  SGPR pairs: CA / BASE the chains' lane masks, SMASK the
        handler's EXEC."""
        assert self.K == 2
        assert not GLIBC4, "glibc_seq3 reads the interleaved table layout"
        cos = want == "cos"
        seq = []
        M = [self.sp(self.CA), self.sp(self.BASE)]
        SV = self.sp(self.SMASK)
        W = "%s_%%=" % want

        def const(name):
            if name in GLIBC_VGPR:
                return "%%[g_%s]" % name.lower()
            i = GLIBC_SGPR.index(name)
            return self.sp((self.TC if i < 8 else self.TC2) + 2 * (i % 8))

        def a(k, t, d=(), u=()):
            t = re.sub(r"@([A-Z0-9_]+)@", lambda m: const(m.group(1)), t)
            seq.append((k, t, tuple(d), tuple(u)))

        def both(t, d=(), u=()):
            for k in range(2):
                a(k, t, d, u)

        def masked(tag, test, d, u, blocks, pre=None):
            """test (per chain, sets VCC) -> the chain's mask; a wave with no
            such lane skips; else blocks(k) under each chain's mask."""
            for k in range(2):
                a(k, test + "\ns_mov_b64 %s, vcc" % M[k], d, u)
            a(1, "s_or_b64 vcc, %s, %s\ns_cbranch_scc0 .L%s_%s" % (M[0], M[1], tag, W))
            if pre:
                pre()
            for k in range(2):
                lab = ".L%s%d_%s" % (tag, k, W)
                a(k, "s_mov_b64 exec, %s\ns_cbranch_execz %s" % (M[k], lab))
                blocks(k)
                a(k, lab + ":")
            a(1, "s_mov_b64 exec, %s\n.L%s_%s:" % (SV, tag, W))

        a(0, "s_mov_b64 %s, exec" % SV)
        if self.prio and not self.prio_late:     # (GEN_ASM_PRIO=tiered: from entry)
            a(0, "s_setprio %d" % self.prio[1])
        # ---- (a, da, n) = (x, 0, sin 0 / cos 1); VRED: max |x|.hi
        both("v_and_b32_e32 {hx}, 0x7fffffff, {x_hi}", ["hx"], ["x"])
        a(1, "v_max3_u32 v%d, v%d, {hx@0}, {hx}" % (self.VRED, self.VRED),
          [], ["hx@0", "hx"])
        # n: bit 31 do_cos (the quadrant's bit 0), bit 0 negate (its bit 1)
        both("v_mov_b64_e32 {da}, 0\n" + ("v_bfrev_b32_e32 {n}, 1" if cos else
                                          "v_mov_b32_e32 {n}, 0"),
             ["da", "n"], [])

        # ---- 0.855469 <= |x| < 2.426265: y = hp0 - |x|; sin: do_cos(y, hp1)
        # with x's sign (n = 1 | sign << 1); cos: do_sin(y + hp1,
        # (y - (y + hp1)) + hp1)
        def dblock(k):
            if cos:
                a(k, "v_add_f64 {y}, @HP0@, -|{x}|", ["y"], ["x"])
                a(k, "v_add_f64 {x}, {y}, @HP1@", [], ["y"])
                a(k, "v_add_f64 {da}, {y}, -{x}", ["da"], ["y", "x", "da"])
                a(k, "v_add_f64 {da}, {da}, @HP1@", ["da"], ["da"])
                a(k, "v_mov_b32_e32 {n}, 0", ["n"], ["n"])
            else:
                a(k, "v_lshrrev_b32_e32 {n}, 31, {x_hi}", ["n"], ["x", "n"])
                a(k, "v_or_b32_e32 {n}, 0x80000000, {n}", ["n"], ["n"])
                a(k, "v_add_f64 {x}, @HP0@, -|{x}|", [], ["x"])
                a(k, "v_mov_b64_e32 {da}, @HP1@", ["da"], ["da"])
        masked("d", "v_subrev_u32_e32 {tm}, 0x3feb6000, {hx}\n"
                    "v_cmp_gt_u32_e32 vcc, 0x%x, {tm}" % (0x400368fd - 0x3feb6000),
               ["tm"], ["hx"], dblock)

        # ---- 2.426265 <= |x| < 105414350: reduce_sincos (n + 1 for cos;
        # only n's low two bits are read)
        def eblock(k):
            a(k, "v_fma_f64 {t}, {x}, @HPINV@, %[mg]", ["t"], ["x"])
            a(k, ("v_add_u32_e32 {n}, 1, {t_lo}\nv_alignbit_b32 {n}, {n}, {n}, 1"
                  if cos else "v_alignbit_b32 {n}, {t_lo}, {t_lo}, 1"),
              ["n"], ["t", "n"])
            a(k, "v_add_f64 {xn}, {t}, -%[mg]", ["xn"], ["t"])
            a(k, "v_fma_f64 {yr}, -{xn}, @MP1@, {x}", ["yr"], ["xn", "x"])
            a(k, "v_fma_f64 {yr}, {xn}, -@MP2@, {yr}", ["yr"], ["xn", "yr"])
            a(k, "v_fma_f64 {t2}, -{xn}, @PP3@, {yr}", ["t2"], ["xn", "yr"])
            a(k, "v_add_f64 {d1}, {yr}, -{t2}", ["d1"], ["yr", "t2"])
            a(k, "v_fma_f64 {db}, -{xn}, @PP3@, {d1}", ["db"], ["xn", "d1"])
            a(k, "v_fma_f64 {x}, -{xn}, @PP4@, {t2}", [], ["xn", "t2"])
            a(k, "v_add_f64 {d2}, {t2}, -{x}", ["d2"], ["t2", "x"])
            a(k, "v_fma_f64 {dar}, -{xn}, @PP4@, {d2}", ["dar"], ["xn", "d2"])
            a(k, "v_add_f64 {da}, {dar}, {db}", ["da"], ["dar", "db", "da"])
        if not ILP:
            masked("e", "v_subrev_u32_e32 {tm}, 0x400368fd, {hx}\n"
                        "v_cmp_gt_u32_e32 vcc, 0x%x, {tm}" % (BRANRED_HI - 0x400368fd),
                   ["tm"], ["hx"], eblock)
        else:
            # both chains' reduce_sincos interleaved (two independent
            # dependency chains) under the union of their masks, into
            # temporaries; then (a, da, n) written under each chain's own
            for k in range(2):
                a(k, "v_subrev_u32_e32 {tm}, 0x400368fd, {hx}\n"
                     "v_cmp_gt_u32_e32 vcc, 0x%x, {tm}\n"
                     "s_mov_b64 %s, vcc" % (BRANRED_HI - 0x400368fd, M[k]),
                  ["tm"], ["hx"])
            a(1, "s_or_b64 exec, %s, %s\ns_cbranch_execz .Le_%s" % (M[0], M[1], W))
            both("v_fma_f64 {t}, {x}, @HPINV@, %[mg]", ["t"], ["x"])
            both("v_add_u32_e32 {nr}, 1, {t_lo}\nv_alignbit_b32 {nr}, {nr}, {nr}, 1"
                 if cos else "v_alignbit_b32 {nr}, {t_lo}, {t_lo}, 1", ["nr"], ["t"])
            both("v_add_f64 {xn}, {t}, -%[mg]", ["xn"], ["t"])
            both("v_fma_f64 {yr}, -{xn}, @MP1@, {x}", ["yr"], ["xn", "x"])
            both("v_fma_f64 {yr}, {xn}, -@MP2@, {yr}", ["yr"], ["xn", "yr"])
            both("v_fma_f64 {t2}, -{xn}, @PP3@, {yr}", ["t2"], ["xn", "yr"])
            both("v_add_f64 {d1}, {yr}, -{t2}", ["d1"], ["yr", "t2"])
            both("v_fma_f64 {db}, -{xn}, @PP3@, {d1}", ["db"], ["xn", "d1"])
            both("v_fma_f64 {b}, -{xn}, @PP4@, {t2}", ["b"], ["xn", "t2"])
            both("v_add_f64 {d2}, {t2}, -{b}", ["d2"], ["t2", "b"])
            both("v_fma_f64 {dar}, -{xn}, @PP4@, {d2}", ["dar"], ["xn", "d2"])
            both("v_add_f64 {dar}, {dar}, {db}", ["dar"], ["dar", "db"])
            for k in range(2):
                a(k, "s_mov_b64 exec, %s\n"
                     "v_mov_b64_e32 {x}, {b}\n"
                     "v_mov_b64_e32 {da}, {dar}\n"
                     "v_mov_b32_e32 {n}, {nr}" % M[k],
                  ["da", "n"], ["b", "dar", "nr", "da", "n"])
            a(1, "s_mov_b64 exec, %s" % SV)
            a(1, ".Le_%s:\ns_mov_b64 exec, %s" % (W, SV))

        # ---- 105414350 <= |x| < inf: __branred (its constants loaded once,
        # under the handler's EXEC)
        keep = {"x", "da", "n", "BK", "bz", "bmp2"}

        def zname(t, vs):
            for v in vs:
                if v not in keep:
                    for sfx in ("", "_lo", "_hi"):
                        t = t.replace("{%s%s}" % (v, sfx), "{z%s%s}" % (v, sfx))
            return t

        def brpre():
            for t, d, u, _ in self.branred_ops(0, want, (self.CA, self.CA + 1))[:4]:
                a(1, zname(t, set(d) | set(u)),
                  [v if v in keep else "z" + v for v in d],
                  [v if v in keep else "z" + v for v in u])

        def brblock(k):
            pair = (self.CA, self.CA + 1) if k == 0 else (self.BASE, self.BASE + 1)
            for t, d, u, _ in self.branred_ops(k, want, pair)[4:]:
                a(k, zname(t, set(d) | set(u)),
                  [v if v in keep else "z" + v for v in d],
                  [v if v in keep else "z" + v for v in u])
        masked("r", "v_subrev_u32_e32 {tm}, 0x%x, {hx}\n"
                    "v_cmp_gt_u32_e32 vcc, 0x%x, {tm}"
               % (BRANRED_HI, 0x7ff00000 - BRANRED_HI),
               ["tm"], ["hx"], brblock, pre=brpre)

        # ---- do_sincos(a, da, n): M[k] = the chain's do_cos lanes (n < 0)
        for k in range(2):
            a(k, "v_cmp_gt_i32_e64 %s, 0, {n}" % M[k], [], ["n"])
        # dx signed as do_sin / do_cos sign it (|a| below), in place: the
        # do_sin lanes' TAYLOR_SIN takes (|a|, that dx) and is odd in (a, da).
        # SCONST = the sign bit; bitop3 0x78: S0 ^ (S1 & S2)
        a(0, "s_brev_b32 s%d, 1" % self.SCONST)
        both("v_bitop3_b32 {da_hi}, {da_hi}, {x_hi}, s%d bitop3:0x78" % self.SCONST,
             ["da"], ["x", "da"])
        both("v_add_f64 {u}, |{x}|, @BIG@", ["u"], ["x"])
        both("v_add_f64 {q1}, {u}, -@BIG@", ["q1"], ["u"])
        both("v_lshlrev_b32_e32 {adr0}, 5, {u_lo}", ["adr0"], ["u"])
        both("v_add_f64 {xr}, |{x}|, -{q1}", ["xr"], ["x", "q1"])
        # (A, Aa, B, Bb) at 32 lo(u): __sincostab, or (do_cos lanes) its
        # cos-ordered copy, SPF bytes on; do_cos lanes: v = xr + dx (into
        # xr), and dx := v (s = v + v xx p)
        for k in range(2):
            lab = ".Lbc%d_%s" % (k, W)
            a(k, "s_mov_b64 exec, %s\ns_cbranch_execz %s" % (M[k], lab))
            a(k, "v_add_u32_e32 {adr0}, s%d, {adr0}" % self.SPF, ["adr0"], ["adr0"])
            a(k, "v_add_f64 {xr}, {xr}, {da}", ["xr"], ["xr", "da"])
            a(k, "v_mov_b64_e32 {da}, {xr}", ["da"], ["xr", "da"])
            a(k, lab + ":")
        a(1, "s_mov_b64 exec, %s" % SV)
        both("v_mul_f64 {xx}, {xr}, {xr}", ["xx"], ["xr"])
        both("v_mul_f64 {m}, {xr}, {xx}", ["m"], ["xr", "xx"])
        both("v_fma_f64 {p}, {xx}, @SN5@, @SN3@", ["p"], ["xx"])
        both("v_fma_f64 {s}, {m}, {p}, {da}", ["s"], ["m", "p", "da"])
        both("v_fma_f64 {w}, {xx}, @CS6@, @CS4@", ["w"], ["xx"])
        both("v_fma_f64 {w}, {w}, {xx}, @CS2@", ["w"], ["w", "xx"])
        both("v_mul_f64 {w}, {w}, {xx}", ["w"], ["w", "xx"])
        both("ds_read_b128 {EA}, {adr0} offset:0", ["EA"], ["adr0"])
        both("ds_read_b128 {EB}, {adr0} offset:16", ["EB"], ["adr0"])
        # do_sin lanes: s = xr + (dx + xr xx p); c = xr dx + w
        for k in range(2):
            lab = ".Lbs%d_%s" % (k, W)
            a(k, "s_andn2_b64 exec, %s, %s\ns_cbranch_execz %s" % (SV, M[k], lab))
            a(k, "v_add_f64 {s}, {s}, {xr}", ["s"], ["s", "xr"])
            a(k, "v_fma_f64 {w}, {da}, {xr}, {w}", ["w"], ["da", "xr", "w"])
            a(k, lab + ":")
        a(1, "s_mov_b64 exec, %s\ns_waitcnt lgkmcnt(0)" % SV)
        if self.prio and self.prio_late:
            a(1, "s_setprio %d" % self.prio[1])
        both("v_fma_f64 {cor}, {s}, {TBb}, {TAa}", ["cor"], ["s", "EB", "EA"])
        both("v_fma_f64 {cor}, -{w}, {TA}, {cor}", ["cor"], ["w", "EA", "cor"])
        both("v_fma_f64 {cor}, {s}, {TB}, {cor}", ["cor"], ["s", "EB", "cor"])
        both("v_add_f64 {r}, {TA}, {cor}", ["r"], ["EA", "cor"])
        # do_sin lanes: |a| < 0.126: TAYLOR_SIN(a a, |a|, dx) (= -TAYLOR_SIN(a
        # a, a, da) for a < 0: every rounding is odd), then copysign(r, a).
        # glibc's |x| < 2^-26 (sin: x) needs no case of its own: there
        # TAYLOR_SIN(x x, |x|, 0) is |x| exactly (|x|^3 / 6 is below half
        # an ulp of |x|, and +0 for +-0), and the copysign restores x
        if not ILP:
            for k in range(2):
                lab = ".Lt%d_%s" % (k, W)
                labc = ".Ltc%d_%s" % (k, W)
                a(k, "s_andn2_b64 exec, %s, %s\ns_cbranch_execz %s" % (SV, M[k], lab))
                a(k, "v_cmp_gt_f64_e64 vcc, @C0126@, |{x}|\n"
                     "s_and_b64 exec, exec, vcc\ns_cbranch_execz %s" % labc, [], ["x"])
                a(k, "v_mul_f64 {xx2}, {x}, {x}", ["xx2"], ["x"])
                a(k, "v_fma_f64 {pt}, {xx2}, @S5@, @S4@", ["pt"], ["xx2"])
                a(k, "v_fma_f64 {pt}, {pt}, {xx2}, @S3@", ["pt"], ["pt", "xx2"])
                a(k, "v_fma_f64 {pt}, {pt}, {xx2}, @S2@", ["pt"], ["pt", "xx2"])
                a(k, "v_fma_f64 {pt}, {pt}, {xx2}, @S1@", ["pt"], ["pt", "xx2"])
                a(k, "v_mul_f64 {h}, {da}, 0.5", ["h"], ["da"])
                a(k, "v_fma_f64 {q}, {pt}, |{x}|, -{h}", ["q"], ["pt", "x", "h"])
                a(k, "v_fma_f64 {q}, {q}, {xx2}, {da}", ["q"], ["q", "xx2", "da"])
                a(k, "v_add_f64 {r}, |{x}|, {q}", ["r"], ["x", "q", "r"])
                a(k, labc + ":\ns_andn2_b64 exec, %s, %s" % (SV, M[k]))
                a(k, "v_bitop3_b32 {r_hi}, {r_hi}, {x_hi}, s%d bitop3:0x78" % self.SCONST,
                  ["r"], ["r", "x"])
                a(k, lab + ":")
            a(1, "s_mov_b64 exec, %s" % SV)
        else:
            # copysign first; then the do_sin lanes' TAYLOR_SIN, both chains
            # interleaved under the union of their masks (M[k] reused), signed
            # in the temporary and written under each chain's own
            for k in range(2):
                lab = ".Lt%d_%s" % (k, W)
                a(k, "s_andn2_b64 exec, %s, %s\ns_mov_b64 %s, 0\n"
                     "s_cbranch_execz %s" % (SV, M[k], M[k], lab))
                a(k, "v_bitop3_b32 {r_hi}, {r_hi}, {x_hi}, s%d bitop3:0x78" % self.SCONST,
                  ["r"], ["r", "x"])
                a(k, "v_cmp_gt_f64_e64 vcc, @C0126@, |{x}|\n"
                     "s_and_b64 %s, exec, vcc\n%s:" % (M[k], lab), [], ["x"])
            a(1, "s_mov_b64 exec, %s" % SV)
            a(1, "s_or_b64 exec, %s, %s\ns_cbranch_execz .Ltt_%s" % (M[0], M[1], W))
            both("v_mul_f64 {xx2}, {x}, {x}", ["xx2"], ["x"])
            both("v_fma_f64 {pt}, {xx2}, @S5@, @S4@", ["pt"], ["xx2"])
            both("v_fma_f64 {pt}, {pt}, {xx2}, @S3@", ["pt"], ["pt", "xx2"])
            both("v_fma_f64 {pt}, {pt}, {xx2}, @S2@", ["pt"], ["pt", "xx2"])
            both("v_fma_f64 {pt}, {pt}, {xx2}, @S1@", ["pt"], ["pt", "xx2"])
            both("v_mul_f64 {h}, {da}, 0.5", ["h"], ["da"])
            both("v_fma_f64 {q}, {pt}, |{x}|, -{h}", ["q"], ["pt", "x", "h"])
            both("v_fma_f64 {q}, {q}, {xx2}, {da}", ["q"], ["q", "xx2", "da"])
            both("v_add_f64 {q}, |{x}|, {q}", ["q"], ["x", "q"])
            both("v_bitop3_b32 {q_hi}, {q_hi}, {x_hi}, s%d bitop3:0x78" % self.SCONST,
                 ["q"], ["q", "x"])
            for k in range(2):
                a(k, "s_mov_b64 exec, %s\nv_mov_b64_e32 {r}, {q}" % M[k], ["r"], ["q", "r"])
            a(1, ".Ltt_%s:\ns_mov_b64 exec, %s" % (W, SV))
        # (n & 2): -r, as an add of n's bit 0 into the sign bit; x = r
        both("v_lshl_add_u32 {x_hi}, {n}, 31, {r_hi}", [], ["n", "r"])
        both("v_mov_b32_e32 {x_lo}, {r_lo}", [], ["r"])
        return seq

    def glibc_seq4(self, want):
        """glibc 2.35 __sin/__cos (gpeval.hip glibc_trig_t) for the K = 2
        chains, every rounding of glibc_seq3's, in fewer VALU instructions
        (round 6; the handler is VALU-issue bound, and every VALU instruction
        costs the SIMD the same four cycles, fp64 or not):

        * ranges: one u32 compare of |x|.hi per threshold (|x| < 0.855469,
          < 2.426265) and SALU masks: d = lt2426 & ~small, e = ~lt2426.  A
          wave none of whose lanes ever held an argument at or past 105414350
          this program (VRED, the running max of |x|.hi, kept anyway for the
          C++ pass's inf/nan test) has no __branred lanes: one compare of
          VRED sends the others to the slow path, which also tests
          < 105414350 and runs __branred (the caller's M0, s81, parked in
          s101 so that s[80:81] is a mask pair there);
        * the do_cos lanes are a mask pair per chain (CA, BASE), formed by
          SALU from those masks (sin: the d lanes, cos: the small ones) plus,
          in the e / __branred blocks, one compare of the quadrant's bit;
        * n (one VGPR per chain, both in one pair: one v_mov_b64 clears them)
          holds only the negation, in bit 31: the d block of sin copies x.hi
          there, reduce_sincos / __branred shift the quadrant to bits 31-30;
          the do_sin lanes fold a's sign in (copysign, as seq3's xor), and
          the result's sign is one bitop3 with it at the end;
        * the result is written into x itself: TAYLOR_SIN's (under its lanes'
          mask, before the table gathers land) and the table path's (under
          the others'), no copies;
        * __sincostab as three 16-byte-stride arrays (A: sn, ssn; B: cs,
          ccs; NA: -sn, -ssn, GLIBC_SPLIT_S apart): a do_sin lane reads A[i]
          and B[i], a do_cos lane B[i] and NA[i] (address + S), so the four
          fma's of the correction are one instruction stream for both.
        SGPRs: CA / BASE the chains' do_cos masks, SMASK the handler's EXEC,
        s80 the sign mask (the slow path: s[80:81] a mask pair), s101 the
        slow path's copy of s81."""
        assert self.K == 2 and GLIBC4
        cos = want == "cos"
        seq = []
        M = [self.sp(self.CA), self.sp(self.BASE)]
        SV = self.sp(self.SMASK)
        SP = self.sp(self.SCONST)
        SC = "s%d" % self.SCONST
        SSAVE = self.SB + 61
        assert self.SCONST + 1 == self.SM0 and SSAVE == 101
        # the compares' threshold register: s101 (the slow path's copy of
        # s81 when M0 lives there), or s80 with M0 in a VGPR lane — then
        # s101 stays free for the loop's window prefetch (GEN_ASM_PF)
        SK = self.SCONST if self.m0lane else SSAVE
        assert not (self.prefetch and not self.m0lane)
        S = GLIBC_SPLIT_S
        W = "%s_%%=" % want
        N = ["{nn_lo}", "{nn_hi}"]

        def const(name):
            if name in GLIBC_VGPR:
                return "%%[g_%s]" % name.lower()
            i = GLIBC_SGPR.index(name)
            return self.sp((self.TC if i < 8 else self.TC2) + 2 * (i % 8))

        def a(k, t, d=(), u=()):
            t = re.sub(r"@([A-Z0-9_]+)@", lambda m: const(m.group(1)), t)
            seq.append((k, t, tuple(d), tuple(u)))

        def both(t, d=(), u=()):
            for k in range(2):
                a(k, t, d, u)

        def dblock(k, pfx):
            """0.855469 <= |x| < 2.426265: y = hp0 - |x|; sin: do_cos(y, hp1)
            negated for x < 0 (n = x.hi); cos: do_sin(y + hp1,
            (y - (y + hp1)) + hp1) (n stays 0)."""
            if cos:
                a(k, "v_add_f64 {%sy}, @HP0@, -|{x}|" % pfx, [pfx + "y"], ["x"])
                a(k, "v_add_f64 {x}, {%sy}, @HP1@" % pfx, [], [pfx + "y"])
                a(k, "v_add_f64 {da}, {%sy}, -{x}" % pfx, ["da"],
                  [pfx + "y", "x", "da"])
                a(k, "v_add_f64 {da}, {da}, @HP1@", ["da"], ["da"])
            else:
                a(k, "v_mov_b32_e32 %s, {x_hi}" % N[k], ["nn"], ["x", "nn"])
                a(k, "v_add_f64 {x}, @HP0@, -|{x}|", [], ["x"])
                a(k, "v_mov_b64_e32 {da}, @HP1@", ["da"], ["da"])

        def eblock(k, pfx):
            """2.426265 <= |x| < 105414350: reduce_sincos; n = the quadrant
            (+1 for cos) << 30; its bit 30 (n as an f32 is +-2.0, else +-0)
            adds the lane to the do_cos mask."""
            z = lambda v: pfx + v
            a(k, "v_fma_f64 {%s}, {x}, @HPINV@, %%[mg]" % z("t"), [z("t")], ["x"])
            a(k, ("v_lshl_add_u32 %s, {%s_lo}, 30, 2.0" if cos else
                  "v_lshlrev_b32_e32 %s, 30, {%s_lo}") % (N[k], z("t")),
              ["nn"], [z("t"), "nn"])
            a(k, "v_add_f64 {%s}, {%s}, -%%[mg]" % (z("xn"), z("t")), [z("xn")], [z("t")])
            a(k, "v_fma_f64 {%s}, -{%s}, @MP1@, {x}" % (z("yr"), z("xn")),
              [z("yr")], [z("xn"), "x"])
            a(k, "v_fma_f64 {%s}, {%s}, -@MP2@, {%s}" % (z("yr"), z("xn"), z("yr")),
              [z("yr")], [z("xn"), z("yr")])
            a(k, "v_fma_f64 {%s}, -{%s}, @PP3@, {%s}" % (z("t2"), z("xn"), z("yr")),
              [z("t2")], [z("xn"), z("yr")])
            a(k, "v_add_f64 {%s}, {%s}, -{%s}" % (z("d1"), z("yr"), z("t2")),
              [z("d1")], [z("yr"), z("t2")])
            a(k, "v_fma_f64 {%s}, -{%s}, @PP3@, {%s}" % (z("db"), z("xn"), z("d1")),
              [z("db")], [z("xn"), z("d1")])
            a(k, "v_fma_f64 {x}, -{%s}, @PP4@, {%s}" % (z("xn"), z("t2")),
              [], [z("xn"), z("t2")])
            a(k, "v_add_f64 {%s}, {%s}, -{x}" % (z("d2"), z("t2")),
              [z("d2")], [z("t2"), "x"])
            a(k, "v_fma_f64 {%s}, -{%s}, @PP4@, {%s}" % (z("dar"), z("xn"), z("d2")),
              [z("dar")], [z("xn"), z("d2")])
            a(k, "v_add_f64 {da}, {%s}, {%s}" % (z("dar"), z("db")), ["da"],
              [z("dar"), z("db"), "da"])
            a(k, "v_cmp_neq_f32_e64 vcc, 0, %s\ns_or_b64 %s, %s, vcc"
              % (N[k], M[k], M[k]), [], ["nn"])

        # ---- |x|.hi (VRED: its running max); M[k] = |x| < 0.855469; the
        # slow-path test; (a, da, n) = (x, 0, 0)
        if not self.salu:
            a(0, "s_mov_b64 %s, exec" % SV)
        if os.environ.get("GEN_ASM_EXPERIMENT") == "dup_salu":
            # (pricing: six more wave-uniform SALU per call, no dependences)
            a(0, "\n".join(["s_mov_b64 %s, exec" % SV] * 6))
        both("v_and_b32_e32 {hx}, 0x7fffffff, {x_hi}", ["hx"], ["x"])
        a(1, "v_max3_u32 v%d, v%d, {hx@0}, {hx}" % (self.VRED, self.VRED),
          [], ["hx@0", "hx"])
        if self.m0lane:
            # the compares straight into their mask pairs (VOP3: the
            # threshold from an SGPR), chain 1's 2.426265 test early (SP)
            if self.salu:                    # (set by the core's prologue)
                assert self.SPF == SSAVE
                for k in range(2):
                    a(k, "v_cmp_gt_u32_e64 %s, s%d, {hx}" % (M[k], SSAVE), [], ["hx"])
            else:
                a(0, "s_mov_b32 s%d, 0x%x" % (SK, GLIBC_T0855))
                for k in range(2):
                    a(k, "v_cmp_gt_u32_e64 %s, s%d, {hx}" % (M[k], SK), [], ["hx"])
            a(1, "s_mov_b32 s%d, 0x400368fd\n"
                 "v_cmp_gt_u32_e64 %s, s%d, {hx}" % (SK, SP, SK), [], ["hx"])
        else:
            for k in range(2):
                a(k, "v_cmp_gt_u32_e32 vcc, 0x3feb6000, {hx}\ns_mov_b64 %s, vcc"
                  % M[k], [], ["hx"])
        a(1, "v_cmp_lt_u32_e32 vcc, 0x%x, v%d" % (BRANRED_HI - 1, self.VRED))
        both("v_mov_b64_e32 {da}, 0", ["da"], [])
        a(0, "v_mov_b64_e32 {nn}, 0", ["nn"], [])
        a(1, "s_cbranch_vccnz .Lslow_%s" % W)
        # ---- fast path (no lane at or past 105414350): per chain, d = lanes
        # below 2.426265 and not small, e = the rest
        for k in range(2):
            lab = "_%d_%s" % (k, W)
            if self.m0lane and k == 1:           # (its test is in SP already)
                a(k, "s_andn2_b64 exec, %s, %s\n"
                     "s_andn2_b64 vcc, %s, %s\n%s"
                     "s_cbranch_execz .Lfd%s" % (SP, M[k], SV, SP, "" if cos else
                                                 "s_mov_b64 %s, exec\n" % M[k], lab))
            else:
                a(k, "v_cmp_gt_u32_e32 vcc, 0x400368fd, {hx}\n"
                     "s_andn2_b64 exec, vcc, %s\n"
                     "s_andn2_b64 vcc, %s, vcc\n%s"
                     "s_cbranch_execz .Lfd%s" % (M[k], SV, "" if cos else
                                                 "s_mov_b64 %s, exec\n" % M[k], lab),
                  [], ["hx"])
            dblock(k, "")
            if self.salu:
                # (SCC: vcc != 0, from the s_andn2 that formed vcc; the d
                # block is VALU only)
                a(k, ".Lfd%s:\ns_cbranch_scc1 .Leo%s" % (lab, lab))
                a(k, "<OOL>\n.Leo%s:\ns_mov_b64 exec, vcc" % lab)
                eblock(k, "")
                a(k, "s_branch .Lfe%s\n<MAIN>" % lab)
            elif OOL:
                # reduce_sincos lanes are rare (17 % of chain-calls): the
                # block sits out of line, the common path falls through
                a(k, ".Lfd%s:\ns_mov_b64 exec, vcc\ns_cbranch_execnz .Leo%s" % (lab, lab))
                a(k, "<OOL>\n.Leo%s:" % lab)
                eblock(k, "")
                a(k, "s_branch .Lfe%s\n<MAIN>" % lab)
            else:
                a(k, ".Lfd%s:\ns_mov_b64 exec, vcc\ns_cbranch_execz .Lfe%s" % (lab, lab))
                eblock(k, "")
            # (the next chain's compares run under the handler's EXEC;
            # with salu, chain 1's first op sets EXEC from its masks)
            if self.salu and k == 0:
                a(k, ".Lfe%s:" % lab)
            else:
                a(k, ".Lfe%s:\ns_mov_b64 exec, %s" % (lab, SV))
        if OOL:
            a(1, "<OOL>")
        else:
            a(1, "s_branch .Ljoin_%s" % W)
        # ---- slow path: the three ranges tested per chain, __branred for the
        # finite lanes at or past 105414350 (its constants loaded once)
        a(1, ".Lslow_%s:" % W if self.m0lane else
          ".Lslow_%s:\ns_mov_b32 s%d, s%d" % (W, SSAVE, self.SM0))
        keep = {"x", "da", "n", "BK", "bz", "bmp2"}

        def brops(k):
            """__branred's ops for chain k: its temporaries renamed (no live
            range shared with the blocks above), n as the chain's half of
            the nn pair, s[80:81] its select pair."""
            out = []
            ren = lambda v: "nn" if v == "n" else v if v in keep else "z" + v
            for t, d, u, _ in self.branred_ops(k, want, (self.SCONST, self.SM0)):
                for v in set(d) | set(u):
                    if v not in keep:
                        for sfx in ("", "_lo", "_hi"):
                            t = t.replace("{%s%s}" % (v, sfx), "{z%s%s}" % (v, sfx))
                t = t.replace("{n}", N[k])
                out.append((t, [ren(v) for v in d], [ren(v) for v in u]))
            return out
        for t, d, u in brops(0)[:4]:          # bz, BK, bmp2 (shared), waited
            a(1, t, d, u)
        for k in range(2):
            lab = "_%d_%s" % (k, W)
            a(k, "v_cmp_gt_u32_e32 vcc, 0x400368fd, {hx}\n"
                 "s_andn2_b64 exec, vcc, %s\n"
                 "s_mov_b64 %s, vcc\n%s"
                 "s_cbranch_execz .Lsd%s" % (M[k], SP, "" if cos else
                                             "s_mov_b64 %s, exec\n" % M[k], lab),
              [], ["hx"])
            dblock(k, "s")
            a(k, ".Lsd%s:\ns_mov_b64 exec, %s\n"
                 "v_cmp_gt_u32_e32 vcc, 0x%x, {hx}\n"
                 "s_andn2_b64 exec, vcc, %s\n"
                 "s_mov_b64 %s, vcc\n"
                 "s_cbranch_execz .Lse%s" % (lab, SV, BRANRED_HI, SP, SP, lab),
              [], ["hx"])
            eblock(k, "s")
            a(k, ".Lse%s:\ns_mov_b64 exec, %s\n"
                 "v_cmp_gt_u32_e32 vcc, 0x7ff00000, {hx}\n"
                 "s_andn2_b64 exec, vcc, %s\n"
                 "s_cbranch_execz .Lsr%s" % (lab, SV, SP, lab), [], ["hx"])
            for t, d, u in brops(k)[4:]:
                a(k, t, d, u)
            a(k, "v_cmp_neq_f32_e64 vcc, 0, %s\ns_or_b64 %s, %s, vcc"
              % (N[k], M[k], M[k]), [], ["nn"])
            a(k, ".Lsr%s:\ns_mov_b64 exec, %s" % (lab, SV))
        restore = "" if self.m0lane else "s_mov_b32 s%d, s%d\n" % (self.SM0, SSAVE)
        if OOL:
            a(1, "%ss_branch .Ljoin_%s\n<MAIN>\n.Ljoin_%s:" % (restore, W, W))
        else:
            a(1, "%s.Ljoin_%s:" % (restore, W))

        # ---- do_sincos(a, da, n): M[k] = the chain's do_cos lanes.  dx
        # signed as do_sin / do_cos sign it (a < 0: -dx), in place: the
        # do_sin lanes' TAYLOR_SIN takes (|a|, that dx) and is odd in (a, da)
        if self.prio and self.prio_late and TRIG_DROP == "join":
            a(0, "s_setprio %d" % self.prio[1])
        a(0, "s_brev_b32 %s, 1" % SC)
        both("v_bitop3_b32 {da_hi}, {da_hi}, {x_hi}, %s bitop3:0x78" % SC,
             ["da"], ["x", "da"])
        both("v_add_f64 {u}, |{x}|, @BIG@", ["u"], ["x"])
        both("v_add_f64 {q1}, {u}, -@BIG@", ["q1"], ["u"])
        both("v_lshlrev_b32_e32 {adr0}, 4, {u_lo}", ["adr0"], ["u"])
        both("v_add_f64 {xr}, |{x}|, -{q1}", ["xr"], ["x", "q1"])
        # do_cos lanes: entries B[i], NA[i]; v = xr + dx (into xr), dx := v
        # (s = v + v xx p)
        for k in range(2):
            lab = ".Lbc%d_%s" % (k, W)
            a(k, "s_mov_b64 exec, %s\ns_cbranch_execz %s" % (M[k], lab))
            a(k, "v_add_u32_e32 {adr0}, 0x%x, {adr0}" % S, ["adr0"], ["adr0"])
            a(k, "v_add_f64 {xr}, {xr}, {da}", ["xr"], ["xr", "da"])
            a(k, "v_mov_b64_e32 {da}, {xr}", ["da"], ["xr", "da"])
            a(k, lab + ":")
        a(1, "s_mov_b64 exec, %s" % SV)
        both("v_mul_f64 {xx}, {xr}, {xr}", ["xx"], ["xr"])
        both("v_mul_f64 {m}, {xr}, {xx}", ["m"], ["xr", "xx"])
        both("v_fma_f64 {p}, {xx}, @SN5@, @SN3@", ["p"], ["xx"])
        both("v_fma_f64 {s}, {m}, {p}, {da}", ["s"], ["m", "p", "da"])
        both("v_fma_f64 {w}, {xx}, @CS6@, @CS4@", ["w"], ["xx"])
        both("v_fma_f64 {w}, {w}, {xx}, @CS2@", ["w"], ["w", "xx"])
        both("v_mul_f64 {w}, {w}, {xx}", ["w"], ["w", "xx"])
        both("ds_read_b128 {EA}, {adr0} offset:0", ["EA"], ["adr0"])
        both("ds_read_b128 {EB}, {adr0} offset:%d" % S, ["EB"], ["adr0"])
        if os.environ.get("GEN_ASM_EXPERIMENT") == "dup_tab":
            # (pricing: a third gather per call and case, same entry, same
            # destination: the values are unchanged)
            both("ds_read_b128 {EB}, {adr0} offset:%d" % S, ["EB"], ["adr0"])
        if self.prio and self.prio_late and TRIG_DROP == "issue":
            a(1, "s_setprio %d" % self.prio[1])
        # do_sin lanes: s = xr + (dx + xr xx p); c = xr dx + w; a's sign
        # into n (copysign, or TAYLOR_SIN's oddness); |a| < 0.126:
        # x = TAYLOR_SIN(a a, |a|, dx) now, and M[k] := the lanes the table
        # result is for (the handler's, less those).  glibc's |x| < 2^-26
        # (sin: x) needs no case of its own: TAYLOR_SIN(x x, |x|, 0) is |x|
        # exactly there (|x|^3 / 6 is below half an ulp; +0 for +-0)
        for k in range(2):
            lab = ".Lbs%d_%s" % (k, W)
            if self.salu:
                # (no do_sin lanes — rare: M := SV out of line; the 0.126
                # compare writes EXEC itself)
                a(k, "s_andn2_b64 exec, %s, %s\ns_cbranch_scc0 .Lns%d_%s"
                  % (SV, M[k], k, W))
                a(k, "<OOL>\n.Lns%d_%s:\ns_mov_b64 %s, %s\ns_branch %s\n<MAIN>"
                  % (k, W, M[k], SV, lab))
            else:
                a(k, "s_andn2_b64 exec, %s, %s\ns_mov_b64 %s, %s\ns_cbranch_scc0 %s"
                  % (SV, M[k], M[k], SV, lab))
            a(k, "v_add_f64 {s}, {s}, {xr}", ["s"], ["s", "xr"])
            a(k, "v_fma_f64 {w}, {da}, {xr}, {w}", ["w"], ["da", "xr", "w"])
            a(k, "v_bitop3_b32 %s, %s, {x_hi}, %s bitop3:0x78" % (N[k], N[k], SC),
              ["nn"], ["nn", "x"])
            if self.salu:
                a(k, "v_cmpx_gt_f64_e64 vcc, @C0126@, |{x}|\n"
                     "s_andn2_b64 %s, %s, exec\n"
                     "s_cbranch_execz %s" % (M[k], SV, lab), [], ["x"])
            else:
                a(k, "v_cmp_gt_f64_e64 vcc, @C0126@, |{x}|\n"
                     "s_and_b64 exec, exec, vcc\n"
                     "s_andn2_b64 %s, %s, exec\n"
                     "s_cbranch_execz %s" % (M[k], SV, lab), [], ["x"])
            a(k, "v_mul_f64 {xx2}, {x}, {x}", ["xx2"], ["x"])
            a(k, "v_fma_f64 {pt}, {xx2}, @S5@, @S4@", ["pt"], ["xx2"])
            a(k, "v_fma_f64 {pt}, {pt}, {xx2}, @S3@", ["pt"], ["pt", "xx2"])
            a(k, "v_fma_f64 {pt}, {pt}, {xx2}, @S2@", ["pt"], ["pt", "xx2"])
            a(k, "v_fma_f64 {pt}, {pt}, {xx2}, @S1@", ["pt"], ["pt", "xx2"])
            a(k, "v_mul_f64 {h}, {da}, 0.5", ["h"], ["da"])
            a(k, "v_fma_f64 {q}, {pt}, |{x}|, -{h}", ["q"], ["pt", "x", "h"])
            a(k, "v_fma_f64 {q}, {q}, {xx2}, {da}", ["q"], ["q", "xx2", "da"])
            a(k, "v_add_f64 {x}, |{x}|, {q}", [], ["x", "q"])
            a(k, lab + ":")
        a(1, "s_mov_b64 exec, %s\ns_waitcnt lgkmcnt(0)" % SV)
        if self.prio and self.prio_late and TRIG_DROP == "wait":
            a(1, "s_setprio %d" % self.prio[1])
        both("v_fma_f64 {cor}, {s}, {TBb}, {TAa}", ["cor"], ["s", "EB", "EA"])
        both("v_fma_f64 {cor}, -{w}, {TA}, {cor}", ["cor"], ["w", "EA", "cor"])
        both("v_fma_f64 {cor}, {s}, {TB}, {cor}", ["cor"], ["s", "EB", "cor"])
        for k in range(2):
            a(k, "s_mov_b64 exec, %s" % M[k])
            a(k, "v_add_f64 {x}, {TA}, {cor}", [], ["EA", "cor", "x"])
        a(1, "s_mov_b64 exec, %s" % SV)
        # the sign: n's bit 31 (negation xor a's sign for do_sin)
        for k in range(2):
            a(k, "v_bitop3_b32 {x_hi}, {x_hi}, %s, %s bitop3:0x78" % (N[k], SC),
              [], ["x", "nn"])
        if os.environ.get("GEN_ASM_EXPERIMENT") == "ulp1":
            # (a deliberately wrong core, for the suite's sensitivity: one ulp
            # added to the ~1/1024 of results whose low 10 bits are zero)
            for k in range(2):
                a(k, "v_and_b32_e32 {ut}, 0x3ff, {x_lo}\n"
                     "v_cmp_eq_u32_e32 vcc, 0, {ut}\n"
                     "v_cndmask_b32_e64 {ut}, 0, 1, vcc\n"
                     "v_add_u32_e32 {x_lo}, {x_lo}, {ut}", ["ut"], ["x"])
        return seq

    def trig_prefix(self, want):
        """If any lane's argument is at or past 2^14 (or nan), branch to the
        mixed body (both reductions, selected per lane): one fp64 compare of
        |x| with 2^14 per case.  sin also goes there for -0.0, the one
        argument the fast body gets wrong (it returns +0.0; tiny nonzero
        arguments come out as x, the correctly rounded sin, as the mixed body
        selects).  The running max of |x|.hi (VRED, the redo test) is only
        kept in the mixed body: the fast body's arguments are below 2^14,
        under every redo threshold.  The inline-constant SGPRs (CA) are free
        in sin/cos handlers, and so is BASE (read by the prologue only): the
        compares write three different pairs before the SALU ORs them, so a
        wave waits on a VALU->SGPR result about once instead of per compare."""
        tests = ["v_cmp_nlt_f64_e64 %%s, |%s|, %s"
                 % (self.p(self.T(k)), self.tc("FAST")) for k in range(self.K)]
        if want == "sin":
            tests += ["v_cmp_class_f64_e64 %%s, %s, 0x20" % self.p(self.T(k))
                      for k in range(self.K)]
        free = [self.sp(self.CA), self.sp(self.BASE), "vcc"]
        pending = []

        def fold():
            a, b = pending.pop(0), pending.pop(0)
            self.e("s_or_b64 %s, %s, %s" % (a, a, b))
            pending.append(a)
            free.append(b)

        for t in tests:
            if not free:
                fold()
            dst = free.pop(0)
            self.e(t % dst)
            pending.append(dst)
        while len(pending) > 1:
            fold()
        self.e("s_and_b64 vcc, exec, %s" % pending[0])
        self.e("s_cbranch_vccnz .Lmix_%s_%%=" % want)

    def vred_update(self):
        """VRED = max(VRED, |x_k|.hi) over the K cases (mixed body).  The
        fast cores track finite arguments only and set bit k of VINF for an
        infinite one (the reference's ValueError at that case, reported by
        the epilogue; a nan argument gives nan either way): neither needs the
        glibc re-run.  The exact core keeps inf/nan in VRED (its C++ pass
        classifies them)."""
        t = self.POOL0
        for k in range(self.K):
            self.e("v_and_b32_e32 v%d, 0x7fffffff, v%d" % (t + k, self.T(k) + 1))
            if not self.exact:
                tmp = t + self.K + k % 2
                if k == 0:                   # NXT is free in sin/cos
                    self.e("s_movk_i32 s%d, 0x204" % self.NXT)       # +-inf
                self.e("v_cmp_class_f64_e64 %s, %s, s%d"
                       % (self.sp(self.CA), self.p(self.T(k)), self.NXT))
                self.e("v_cndmask_b32_e64 v%d, 0, %d, %s"
                       % (tmp, 1 << k, self.sp(self.CA)))
                self.e("v_or_b32_e32 v%d, v%d, v%d" % (self.VINF, self.VINF, tmp))
                self.e("v_cmp_gt_u32_e32 vcc, 0x7ff00000, v%d" % (t + k))
                self.e("v_cndmask_b32_e32 v%d, 0, v%d, vcc" % (t + k, t + k))
        self.use_v(t + self.K + 2)
        for k in range(0, self.K - 1, 2):          # max3 takes two at a time
            self.e("v_max3_u32 v%d, v%d, v%d, v%d"
                   % (self.VRED, self.VRED, t + k, t + k + 1))
        if self.K % 2:
            self.e("v_max_u32_e32 v%d, v%d, v%d"
                   % (self.VRED, self.VRED, t + self.K - 1))

    def branred_ops(self, k, want, pair=None):
        """glibc's __branred (gpeval.hip glibc::branred, branred.c) for case
        k's lanes with 105414350 <= |x| < inf, as ops like glibc_ops: x
        scaled by 2^-600 and split in two 27-bit halves; per half, six
        products with the 24-bit digits of 2/pi (toverp, LDS) scaled by
        2^(576 - 24 k - 24 i) (ldexp: exact, as glibc's power-of-two gor),
        the integer parts peeled off with the 1.5 * 2^52 (%[mg]) and
        1.5 * 2^54 roundings; the halves combined and multiplied by pi/2 in
        double-double.  No fma anywhere (the library's C++ is built with
        -ffp-contract=off and matches the host libm bit for bit).  Other
        lanes compute garbage (toverp index clamped) and keep their (a, da,
        n); the quadrant gets +1 for cos."""
        ops = []

        def op(t, d=(), u=()):
            ops.append((t, tuple(d), tuple(u), False))
        cst = GLIBC_BRANRED_BYTES              # SPLIT, BBIG1, BMP2 in LDS
        tov = cst + 32                         # toverp[0]
        sp = lambda n: self.sp(n)
        HP0, HP1, MP1 = (self.sp((self.TC if GLIBC_SGPR.index(c) < 8 else self.TC2)
                                 + 2 * (GLIBC_SGPR.index(c) % 8))
                         for c in ("HP0", "HP1", "MP1"))
        op("v_mov_b32_e32 {bz}, 0", ["bz"], [])
        op("ds_read_b128 {BK}, {bz} offset:%d" % cst, ["BK"], ["bz"])
        op("ds_read_b64 {bmp2}, {bz} offset:%d" % (cst + 16), ["bmp2"], ["bz"])
        op("s_waitcnt lgkmcnt(0)", [], [])
        # x *= 2^-600 (exact); t = x * SPLIT; x1 = t - (t - x); x2 = x - x1
        op("s_movk_i32 s%d, 0xfda8" % self.NXT)          # -600
        op("v_ldexp_f64 {xs}, {x}, s%d" % self.NXT, ["xs"], ["x"])
        op("v_mul_f64 {bt}, {xs}, {bsplit}", ["bt"], ["xs", "BK"])
        op("v_add_f64 {bu}, {bt}, -{xs}", ["bu"], ["bt", "xs"])
        op("v_add_f64 {x1}, {bt}, -{bu}", ["x1"], ["bt", "bu"])
        op("v_add_f64 {x2}, {xs}, -{x1}", ["x2"], ["xs", "x1"])
        for h in ("1", "2"):
            xh = "x" + h
            b, sm, bb = "b" + h, "sum" + h, "bb" + h
            # k = max(e - 450, 0) / 24 (<= 69: garbage lanes); the exponent
            # of gor_i = 576 - 24 k - 24 i
            op("v_bfe_u32 {e}, {%s_hi}, 20, 11" % xh, ["e"], [xh])
            op("v_subrev_u32_e32 {e}, 0x1c2, {e}", ["e"], ["e"])
            op("v_max_i32_e32 {e}, 0, {e}", ["e"], ["e"])
            op("s_mov_b32 s%d, 0xaaaaaaab" % self.NXT)
            op("v_mul_hi_u32 {e}, {e}, s%d" % self.NXT, ["e"], ["e"])
            op("v_lshrrev_b32_e32 {e}, 4, {e}", ["e"], ["e"])
            op("v_min_u32_e32 {e}, 0x45, {e}", ["e"], ["e"])
            op("v_lshlrev_b32_e32 {adr}, 3, {e}", ["adr"], ["e"])
            op("v_mul_u32_u24_e32 {e}, 24, {e}", ["e"], ["e"])
            op("v_sub_u32_e32 {e}, 0x240, {e}", ["e"], ["e"])
            for i in range(6):
                op("ds_read_b64 {r%d}, {adr} offset:%d" % (i, tov + 8 * i),
                   ["r%d" % i], ["adr"])
            op("s_waitcnt lgkmcnt(0)", [], [])
            for i in range(6):
                op("v_mul_f64 {r%d}, {%s}, {r%d}" % (i, xh, i), ["r%d" % i],
                   [xh, "r%d" % i])
                if i:
                    op("v_subrev_u32_e32 {ei}, %d, {e}" % (24 * i), ["ei"], ["e"])
                    op("v_ldexp_f64 {r%d}, {r%d}, {ei}" % (i, i), ["r%d" % i],
                       ["r%d" % i, "ei"])
                else:
                    op("v_ldexp_f64 {r0}, {r0}, {e}", ["r0"], ["r0", "e"])
            # sum = 0; 3 x: s = (r[i] + BBIG) - BBIG; sum += s; r[i] -= s
            for i in range(3):
                r = "r%d" % i
                op("v_add_f64 {s}, {%s}, %%[mg]" % r, ["s"], [r])
                op("v_add_f64 {s}, {s}, -%[mg]", ["s"], ["s"])
                if i == 0:
                    op("v_add_f64 {%s}, 0, {s}" % sm, [sm], ["s"])
                else:
                    op("v_add_f64 {%s}, {%s}, {s}" % (sm, sm), [sm], [sm, "s"])
                op("v_add_f64 {%s}, {%s}, -{s}" % (r, r), [r], [r, "s"])
            # t = 0; t += r[5 - i]; bb = (((((r0 - t) + r1) + r2) + r3) + r4) + r5
            op("v_add_f64 {tt}, 0, {r5}", ["tt"], ["r5"])
            for i in (4, 3, 2, 1, 0):
                op("v_add_f64 {tt}, {tt}, {r%d}" % i, ["tt"], ["tt", "r%d" % i])
            op("v_add_f64 {w}, {r0}, -{tt}", ["w"], ["r0", "tt"])
            for i in range(1, 6):
                op("v_add_f64 {w}, {w}, {r%d}" % i, ["w"], ["w", "r%d" % i])
            # s = (t + BBIG) - BBIG; sum += s; t -= s; b = t + bb;
            # bb = (t - b) + bb; s = (sum + BBIG1) - BBIG1; sum -= s
            op("v_add_f64 {s}, {tt}, %[mg]", ["s"], ["tt"])
            op("v_add_f64 {s}, {s}, -%[mg]", ["s"], ["s"])
            op("v_add_f64 {%s}, {%s}, {s}" % (sm, sm), [sm], [sm, "s"])
            op("v_add_f64 {tt}, {tt}, -{s}", ["tt"], ["tt", "s"])
            op("v_add_f64 {%s}, {tt}, {w}" % b, [b], ["tt", "w"])
            op("v_add_f64 {tt}, {tt}, -{%s}" % b, ["tt"], ["tt", b])
            op("v_add_f64 {%s}, {tt}, {w}" % bb, [bb], ["tt", "w"])
            op("v_add_f64 {s}, {%s}, {bbig1}" % sm, ["s"], [sm, "BK"])
            op("v_add_f64 {s}, {s}, -{bbig1}", ["s"], ["s", "BK"])
            op("v_add_f64 {%s}, {%s}, -{s}" % (sm, sm), [sm], [sm, "s"])
        # sum = sum1 + sum2; b = b1 + b2;
        # bb = |b1| > |b2| ? (b1 - b) + b2 : (b2 - b) + b1
        op("v_add_f64 {sum}, {sum1}, {sum2}", ["sum"], ["sum1", "sum2"])
        op("v_add_f64 {b}, {b1}, {b2}", ["b"], ["b1", "b2"])
        op("v_add_f64 {p1}, {b1}, -{b}", ["p1"], ["b1", "b"])
        op("v_add_f64 {p1}, {p1}, {b2}", ["p1"], ["p1", "b2"])
        op("v_add_f64 {p2}, {b2}, -{b}", ["p2"], ["b2", "b"])
        op("v_add_f64 {p2}, {p2}, {b1}", ["p2"], ["p2", "b1"])
        op("v_cmp_gt_f64_e64 vcc, |{b1}|, |{b2}|\n"
           "v_cndmask_b32_e32 {bb_lo}, {p2_lo}, {p1_lo}, vcc\n"
           "v_cndmask_b32_e32 {bb_hi}, {p2_hi}, {p1_hi}, vcc",
           ["bb"], ["b1", "b2", "p1", "p2"])
        # b > 0.5: b -= 1, sum += 1; b < -0.5: b += 1, sum -= 1
        op("v_add_f64 {p1}, {b}, -1.0", ["p1"], ["b"])
        op("v_add_f64 {p2}, {sum}, 1.0", ["p2"], ["sum"])
        op("v_add_f64 {q1}, {b}, 1.0", ["q1"], ["b"])
        op("v_add_f64 {q2}, {sum}, -1.0", ["q2"], ["sum"])
        op("v_cmp_lt_f64_e32 vcc, 0.5, {b}\n"
           "v_cndmask_b32_e32 {sum_lo}, {sum_lo}, {p2_lo}, vcc\n"
           "v_cndmask_b32_e32 {sum_hi}, {sum_hi}, {p2_hi}, vcc\n"
           "v_cmp_gt_f64_e64 s[%d:%d], -0.5, {b}\n"
           "v_cndmask_b32_e32 {b_lo}, {b_lo}, {p1_lo}, vcc\n"
           "v_cndmask_b32_e32 {b_hi}, {b_hi}, {p1_hi}, vcc\n"
           "v_cndmask_b32_e64 {sum_lo}, {sum_lo}, {q2_lo}, s[%d:%d]\n"
           "v_cndmask_b32_e64 {sum_hi}, {sum_hi}, {q2_hi}, s[%d:%d]\n"
           "v_cndmask_b32_e64 {b_lo}, {b_lo}, {q1_lo}, s[%d:%d]\n"
           "v_cndmask_b32_e64 {b_hi}, {b_hi}, {q1_hi}, s[%d:%d]"
           % ((pair or (self.SMASK, self.SMASK + 1)) * 5),
           ["sum", "b"], ["sum", "b", "p1", "p2", "q1", "q2"])
        # s = b + ((bb + bb1) + bb2); t = ((b - s) + bb) + (bb1 + bb2)
        op("v_add_f64 {w}, {bb}, {bb1}", ["w"], ["bb", "bb1"])
        op("v_add_f64 {w}, {w}, {bb2}", ["w"], ["w", "bb2"])
        op("v_add_f64 {s}, {b}, {w}", ["s"], ["b", "w"])
        op("v_add_f64 {tt}, {b}, -{s}", ["tt"], ["b", "s"])
        op("v_add_f64 {tt}, {tt}, {bb}", ["tt"], ["tt", "bb"])
        op("v_add_f64 {w}, {bb1}, {bb2}", ["w"], ["bb1", "bb2"])
        op("v_add_f64 {tt}, {tt}, {w}", ["tt"], ["tt", "w"])
        # b = s * SPLIT; t1 = b - (b - s); t2 = s - t1; b = s * hp0
        op("v_mul_f64 {q1}, {s}, {bsplit}", ["q1"], ["s", "BK"])
        op("v_add_f64 {q2}, {q1}, -{s}", ["q2"], ["q1", "s"])
        op("v_add_f64 {t1}, {q1}, -{q2}", ["t1"], ["q1", "q2"])
        op("v_add_f64 {t2}, {s}, -{t1}", ["t2"], ["s", "t1"])
        op("v_mul_f64 {b}, {s}, %s" % HP0, ["b"], ["s"])
        # bb = (((t1 mp1 - b) + t1 bmp2) + t2 mp1) + (t2 bmp2 + s hp1 + t hp0)
        op("v_mul_f64 {p1}, {t1}, %s" % MP1, ["p1"], ["t1"])
        op("v_add_f64 {p1}, {p1}, -{b}", ["p1"], ["p1", "b"])
        op("v_mul_f64 {p2}, {t1}, {bmp2}", ["p2"], ["t1", "bmp2"])
        op("v_add_f64 {p1}, {p1}, {p2}", ["p1"], ["p1", "p2"])
        op("v_mul_f64 {p2}, {t2}, %s" % MP1, ["p2"], ["t2"])
        op("v_add_f64 {p1}, {p1}, {p2}", ["p1"], ["p1", "p2"])
        op("v_mul_f64 {q1}, {t2}, {bmp2}", ["q1"], ["t2", "bmp2"])
        op("v_mul_f64 {q2}, {s}, %s" % HP1, ["q2"], ["s"])
        op("v_add_f64 {q1}, {q1}, {q2}", ["q1"], ["q1", "q2"])
        op("v_mul_f64 {q2}, {tt}, %s" % HP0, ["q2"], ["tt"])
        op("v_add_f64 {q1}, {q1}, {q2}", ["q1"], ["q1", "q2"])
        op("v_add_f64 {p1}, {p1}, {q1}", ["p1"], ["p1", "q1"])
        # a = b + bb; da = (b - a) + bb; n = ((int) sum & 3) (+1: cos)
        if pair is not None:             # under the chain's exec mask
            op("v_add_f64 {x}, {b}, {p1}", [], ["b", "p1"])
            op("v_add_f64 {da}, {b}, -{x}", ["da"], ["b", "x", "da"])
            op("v_add_f64 {da}, {da}, {p1}", ["da"], ["da", "p1"])
            op("v_cvt_i32_f64_e32 {n}, {sum}", ["n"], ["sum", "n"])
            if want == "cos":
                op("v_add_u32_e32 {n}, 1, {n}", ["n"], ["n"])
            if GLIBC4:
                # glibc_seq4's n: the quadrant's two bits at the top (bit 31:
                # negate, bit 30: do_cos)
                op("v_lshlrev_b32_e32 {n}, 30, {n}", ["n"], ["n"])
            else:
                # glibc_seq3's n: the quadrant rotated right by one (bit 31:
                # do_cos, bit 0: negate)
                op("v_alignbit_b32 {n}, {n}, {n}, 1", ["n"], ["n"])
            return ops
        op("v_add_f64 {q1}, {b}, {p1}", ["q1"], ["b", "p1"])
        op("v_add_f64 {q2}, {b}, -{q1}", ["q2"], ["b", "q1"])
        op("v_add_f64 {q2}, {q2}, {p1}", ["q2"], ["q2", "p1"])
        op("v_cvt_i32_f64_e32 {nb}, {sum}", ["nb"], ["sum"])
        op("v_and_b32_e32 {nb}, 3, {nb}", ["nb"], ["nb"])
        if want == "cos":
            op("v_add_u32_e32 {nb}, 1, {nb}", ["nb"], ["nb"])
        op("v_subrev_u32_e32 {tm}, 0x%x, {hx}\n"
           "v_cmp_gt_u32_e32 vcc, 0x%x, {tm}\n"
           "v_cndmask_b32_e32 {a_lo}, {a_lo}, {q1_lo}, vcc\n"
           "v_cndmask_b32_e32 {a_hi}, {a_hi}, {q1_hi}, vcc\n"
           "v_cndmask_b32_e32 {da_lo}, {da_lo}, {q2_lo}, vcc\n"
           "v_cndmask_b32_e32 {da_hi}, {da_hi}, {q2_hi}, vcc\n"
           "v_cndmask_b32_e32 {n}, {n}, {nb}, vcc"
           % (BRANRED_HI, 0x7ff00000 - BRANRED_HI),
           ["tm", "a", "da", "n"], ["hx", "a", "da", "n", "q1", "q2", "nb"])
        return ops

    def branred_block(self, want, ks, tag):
        """The seq entries of the __branred block for chains ks: a wave with
        any such lane (105414350 <= |x| < inf) in any of them runs it."""
        seq = []
        for j, k in enumerate(ks):
            seq.append((k, "v_subrev_u32_e32 {tm}, 0x%x, {hx}\n"
                           "v_cmp_gt_u32_e32 vcc, 0x%x, {tm}\n"
                           "s_%s_b64 s[%d:%d], %svcc"
                        % (BRANRED_HI, 0x7ff00000 - BRANRED_HI,
                           "mov" if j == 0 else "or", self.CA, self.CA + 1,
                           "" if j == 0 else "s[%d:%d], " % (self.CA, self.CA + 1)),
                        ("tm",), ("hx",)))
        label = ".Lnobr_%s_%s_%%=" % (want, tag)
        seq.append((ks[0], "s_and_b64 vcc, exec, s[%d:%d]\ns_cbranch_vccz %s"
                    % (self.CA, self.CA + 1, label), (), ()))
        keep = {"x", "a", "da", "n", "hx", "tm", "BK", "bz", "bmp2"}

        def z(v):                # the block's own names: no live range is
            return v if v in keep else "z" + v   # shared with glibc_ops's
        for j, k in enumerate(ks):
            ops = self.branred_ops(k, want)
            if j:                    # the constants: loaded once
                ops = ops[4:]
            for t, d, u, _ in ops:
                for v in set(d) | set(u):
                    if v not in keep:
                        for sfx in ("", "_lo", "_hi"):
                            t = t.replace("{%s%s}" % (v, sfx), "{z%s%s}" % (v, sfx))
                seq.append((k, t, tuple(z(v) for v in d), tuple(z(v) for v in u)))
        seq.append((ks[0], label + ":", (), ()))
        return seq

    def sincos(self, want, mixed=False):
        """The K chains of gp_trig, registers linear-scan allocated from the
        temporary pool: interleaved instruction by instruction in the fast
        body; one after the other in the (rare) mixed body, which keeps its
        temporaries — and so the core's VGPR count — down.  A chain's own
        two table reads are the youngest LDS operations at its waits."""
        K = self.K
        if self.exact and GLIBC4 and not mixed:
            self._alloc_emit(self.glibc_seq4(want))
            return
        if self.exact and GLIBC3 and not mixed:
            self._alloc_emit(self.glibc_seq3(want))
            return
        gops = self.glibc_ops2 if GLIBC2 else self.glibc_ops
        chains = [gops(k, want) if self.exact else
                  self.trig_ops(k, want, mixed) for k in range(K)]
        n = len(chains[0])
        # fast body: the chains interleaved G at a time (G = K: all of them;
        # a smaller group keeps the temporaries, and so the VGPRs, of a
        # many-case core down)
        G = 1 if mixed else min(K, self.trig_group or K)
        groups = [list(range(g, min(K, g + G))) for g in range(0, K, G)]
        order = [(k, i) for grp in groups for i in range(n) for k in grp]
        grp_of = {k: grp for grp in groups for k in grp}
        nout = (4 if SPLIT_TAB and not self.exact else 2) * G   # table reads
        if os.environ.get("GEN_ASM_EXPERIMENT") == "dup_tab" and not self.exact:
            nout = 3 * G
        seq = []                       # (k, template, defs, uses)
        for k, i in order:
            t, d, u, once = chains[k][i]
            if once == "branred":          # after the chains' reductions
                grp = [k] if mixed else next(g for g in groups if k in g)
                if k == grp[-1]:
                    seq.extend(self.branred_block(want, grp, "%d" % grp[0]))
                continue
            if once in ("rskip_beg", "rskip_end"):
                # the exact core's wave-uniform skip of reduce_sincos: each
                # chain compares its |x| with 2.426265 (the pair CA, free in
                # sin/cos handlers, gathers both), the last one branches past
                # the block when every active lane of both is below
                if not (self.rskip and G == K == 2):
                    continue
                lab = ".Lrskip_%s_%%=" % want
                if once == "rskip_beg":
                    # (VOPC takes the literal; VOP3 would not: via VCC)
                    ca = self.sp(self.CA)
                    lines = ["v_cmp_gt_u32_e32 vcc, 0x400368fd, {hx}"]
                    if k == 0:
                        lines.append("s_mov_b64 %s, vcc" % ca)
                    else:
                        lines += ["s_and_b64 %s, %s, vcc" % (ca, ca),
                                  "s_andn2_b64 %s, exec, %s" % (ca, ca),
                                  "s_cbranch_scc0 %s" % lab]
                    seq.append((k, "\n".join(lines), (), ("hx",)))
                elif k == K - 1:
                    seq.append((k, lab + ":", (), ()))
                continue
            if isinstance(once, tuple):
                # glibc_ops2's control flow (chains interleaved: the block
                # tests accumulate over the chains, the last one branches)
                kind = once[0]
                last = k == grp_of[k][-1]
                if kind == "need":
                    pair = once[1]
                    acc = ("s_mov_b64 %s, vcc" % pair if k == grp_of[k][0]
                           else "s_or_b64 %s, %s, vcc" % (pair, pair))
                    seq.append((k, t + "\n" + acc, d, u))
                elif kind == "skipto" and last:
                    seq.append((k, "s_and_b64 %s, exec, %s\ns_cbranch_scc0 %s"
                                % (once[1], once[1], once[2]), (), ()))
                elif kind == "label" and last:
                    seq.append((k, once[1] + ":", (), ()))
                elif kind == "once" and last:
                    seq.append((k, t, d, u))
                continue
            if once == "wait":
                if k % G and not mixed:
                    continue
                t = t.replace("@NOUT@", str(nout))
            elif once and k:
                continue
            seq.append((k, t, d, u))
        self._alloc_emit(seq)

    def _alloc_emit(self, seq):
        """Linear-scan register allocation of a sin/cos seq — (chain,
        template, defs, uses) entries, {name} fields, a use "v@k" naming
        chain k's v — and emission."""
        singles = {"ax", "ax2", "j", "cadr", "hx", "tm", "nr", "n", "nm", "sa", "ut",
                   "isc", "flip", "sg", "adr", "adr2", "sgn", "rc", "ng", "bz", "ze",
                   "zei", "znb", "zadr"}
        quads = {"SQ", "CQ", "CL", "E0", "E1", "BK", "EA", "EB"} | \
            {q + "_" + kd for q in ("EA", "EB") for kd in "msc"}
        singles |= {"adr_" + kd for kd in "msc"} | {"adr0"}
        # one copy for all chains
        shared = {"cadr", "CL", "bz", "BK", "bmp2", "nn"}
        halves = {"SQ": ("sh", "sl"), "CQ": ("ch", "cl"), "CL": ("c2", "c3"),
                  "E0": ("sn", "ssn"), "E1": ("cs", "ccs"),
                  "EA_m": ("TA_m", "TAa_m"), "EB_m": ("TB_m", "TBb_m"),
                  "EA_s": ("TA_s", "TAa_s"), "EB_s": ("TB_s", "TBb_s"),
                  "EA_c": ("TA_c", "TAa_c"), "EB_c": ("TB_c", "TBb_c"),
                  "BK": ("bsplit", "bbig1"), "EA": ("TA", "TAa"),
                  "EB": ("TB", "TBb")}

        def kk(k, v):
            if "@" in v:
                v, k = v.split("@")
                k = int(k)
            return (0, v) if v in shared else (k, v)

        def vbase(v):
            return v.split("@")[0]
        last = {}
        for idx, (k, t, d, u) in enumerate(seq):
            for v in u:
                last[kk(k, v)] = idx
        for idx, (k, t, d, u) in enumerate(seq):
            for v in d:
                last.setdefault(kk(k, v), idx)
        free1, free2 = [], []          # free single VGPRs / free pairs
        nxt = [self.POOL0]             # next never-used VGPR

        def get(kind):
            if kind == 1:
                if free1:
                    return free1.pop(0)
                if free2:
                    r = free2.pop(0)
                    free1.append(r + 1)
                    return r
                r = nxt[0]
                nxt[0] += 2
                free1.append(r + 1)
                return r
            if kind == 2:
                if free2:
                    return free2.pop(0)
                r = nxt[0]
                nxt[0] += 2
                return r
            # quad, 4-aligned: two free adjacent pairs, else fresh registers
            for r in free2:
                if r % 4 == 0 and r + 2 in free2:
                    free2.remove(r)
                    free2.remove(r + 2)
                    return r
            if nxt[0] % 4:
                free2.append(nxt[0])
                nxt[0] += 2
            r = nxt[0]
            nxt[0] += 4
            return r

        def put(v, r):
            v = vbase(v)
            if v in singles:
                free1.append(r)
            elif v in quads:
                free2.extend([r, r + 2])
            else:
                free2.append(r)
            free1.sort()
            free2.sort()

        where = {}

        def name(names, v, r):
            if vbase(v) in singles:
                names[v] = "v%d" % r
            elif vbase(v) in quads:
                names[v] = "v[%d:%d]" % (r, r + 3)
                lo, hi = halves[v]
                names[lo] = self.p(r)
                names[hi] = self.p(r + 2)
                for h, base in ((lo, r), (hi, r + 2)):
                    names[h + "_lo"] = "v%d" % base
                    names[h + "_hi"] = "v%d" % (base + 1)
            else:
                names[v] = self.p(r)
                names[v + "_lo"] = "v%d" % r
                names[v + "_hi"] = "v%d" % (r + 1)

        for idx, (k, t, d, u) in enumerate(seq):
            multi = "\n" in t
            names = {"x": self.p(self.T(k)), "x_lo": "v%d" % self.T(k),
                     "x_hi": "v%d" % (self.T(k) + 1)}
            for v in u:
                if v != "x":
                    name(names, v, where[kk(k, v)])
            dying = [v for v in set(u) if v != "x" and last[kk(k, v)] == idx]
            if not multi:                # srcs dying here may be reused
                for v in dying:
                    put(v, where.pop(kk(k, v)))
            for v in d:
                key = kk(k, v)
                if key not in where:
                    kind = 1 if v in singles else 4 if v in quads else 2
                    where[key] = get(kind)
                name(names, v, where[key])
            if multi:
                for v in dying:
                    put(v, where.pop(kk(k, v)))
            for line in t.split("\n"):
                if line in ("<OOL>", "<MAIN>"):      # emission section switch
                    self._in_ool = line == "<OOL>"
                    continue
                self.e(line.format(**names) if "{" in line else line)
            # drop defs that are never used (dead results)
            for v in d:
                key = kk(k, v)
                if key in where and last[key] == idx:
                    put(v, where.pop(key))
        self.use_v(nxt[0] - 1)

    # ------------------------------------------------------ program loop --
    def loop_next(self):
        """.Lnext: start program %[jio] of the wave (lane j of %[vstart]
        holds its first code word), or leave with %[jio] = %[nmine] once
        the wave's programs are done; programs whose bit is set in %[done]
        (re-run whole with glibc's sin/cos) are skipped."""
        W, NX = self.WIN, self.NXT
        self.e("s_nop 4")              # the caller's writes of the inputs
        self.label(".Lnext_")
        self.e("s_cmp_ge_u32 s%d, %%[nmine]" % self.SJ)
        self.e("s_cbranch_scc1 .Lend_%=")
        self.e("s_bitcmp1_b32 %%[done], s%d" % self.SJ)
        self.e("s_cbranch_scc1 .Lskip_%=")
        if self.prefetch:
            # END already loaded this program's first window (and waited)
            self.e("s_cmp_eq_u32 s%d, s%d" % (self.SPF, self.SJ))
            self.e("s_cbranch_scc1 .Lhave_%=")
        self.load_first_window(self.SJ)
        self.label(".Lhave_")
        if self.prefetch:
            self.e("s_mov_b32 s%d, -1" % self.SPF)
        self.e("v_mov_b32_e32 v%d, 0" % self.VRED)
        if not self.exact:
            self.e("v_mov_b32_e32 v%d, 0" % self.VINF)
        self.e("s_mov_b32 m0, 0")
        self.e("s_waitcnt lgkmcnt(0)")
        self.e("s_nop 0")
        self.dispatch_head()
        self.dispatch_tail()
        self.label(".Lskip_")
        if self.prefetch:
            # a window prefetched for this skipped program must land before
            # the next load into the same SGPRs (or the core's exit)
            self.e("s_waitcnt lgkmcnt(0)")
        self.e("s_add_u32 s%d, s%d, 1" % (self.SJ, self.SJ))
        self.e("s_branch .Lnext_%=")

    def load_first_window(self, sj):
        """s[WIN..] = the first window of program s<sj> of the wave (lane
        s<sj> of %[vstart] holds its first code word); PTR its address."""
        W, NX = self.WIN, self.NXT
        self.e("v_readlane_b32 s%d, %%[vstart], s%d" % (NX, sj))
        self.e("s_nop 4")
        self.e("s_lshl_b32 s%d, s%d, 2" % (NX, NX))
        self.e("s_add_u32 s%d, %%[code_lo], s%d" % (self.PTR, NX))
        self.e("s_addc_u32 s%d, %%[code_hi], 0" % (self.PTR + 1))
        self.e("s_load_dwordx16 s[%d:%d], %s, 0x0"
               % (W, W + 15, self.sp(self.PTR)))

    def loop_end(self):
        """END of a program in the loop core: the caller finishes it (leave
        with T, VRED, VINF and %[jio] = its index) if the tile is not lean
        (%[lean] = 0), an argument asked for the glibc re-run (VRED at or
        past %[rhi]), an argument was infinite (VINF) or the sum is not
        finite; else the lean MSE epilogue of f_eval_asm, operation for
        operation: d = T - y, d*d, TwoSum into the program's (hi, lo) at
        LDS %[vacc] + 1024 j (lo 512 on), y at %[vts] + 512 k."""
        K, P = self.K, self.p
        self.e("s_cmp_eq_u32 %[lean], 0")
        self.e("s_cbranch_scc1 .Lend_%=")
        self.e("v_cmp_le_u32_e64 vcc, %%[rhi], v%d" % self.VRED)
        self.e("s_and_b64 vcc, exec, vcc")
        self.e("s_cbranch_vccnz .Lend_%=")
        if not self.exact:             # (the exact core keeps inf in VRED)
            self.e("v_cmp_ne_u32_e32 vcc, 0, v%d" % self.VINF)
            self.e("s_and_b64 vcc, exec, vcc")
            self.e("s_cbranch_vccnz .Lend_%=")
        b = self.POOL0
        Y = [b + 2 * k for k in range(K)]
        HI, LO = b + 2 * K, b + 2 * K + 2
        A = b + 2 * K + 4                      # address (one VGPR, pair slot)
        NS, BB, T1, T2 = [b + 2 * K + 6 + 2 * i for i in range(4)]
        SQ = [T2 + 2 + 2 * k for k in range(K)]
        self.use_v(SQ[-1] + 1)
        if self.read2 and K == 2:
            self.e("ds_read2st64_b64 v[%d:%d], %%[vts] offset0:0 offset1:1"
                   % (Y[0], Y[0] + 3))
        else:
            for k in range(K):
                self.e("ds_read_b64 %s, %%[vts] offset:%d" % (P(Y[k]), 512 * k))
        self.e("s_lshl_b32 s%d, s%d, 10" % (self.NXT, self.SJ))
        self.e("v_add_u32_e32 v%d, s%d, %%[vacc]" % (A, self.NXT))
        if self.read2:
            assert LO == HI + 2
            self.e("ds_read2st64_b64 v[%d:%d], v%d offset0:0 offset1:1"
                   % (HI, HI + 3, A))
        else:
            self.e("ds_read_b64 %s, v%d" % (P(HI), A))
            self.e("ds_read_b64 %s, v%d offset:512" % (P(LO), A))
        if self.prefetch:
            # the next program's first window, loaded while these LDS reads
            # are in flight (the window SGPRs are dead at END; one wait for
            # both: the load's latency no longer follows the epilogue)
            self.e("s_add_u32 s%d, s%d, 1" % (self.SPF, self.SJ))
            self.e("s_cmp_lt_u32 s%d, %%[nmine]" % self.SPF)
            self.e("s_cbranch_scc0 .Lnopf_%=")
            self.load_first_window(self.SPF)
            self.label(".Lnopf_")
        self.e("s_waitcnt lgkmcnt(0)")
        # dlt = T - y and sq = dlt*dlt for every case first (independent),
        # then the running (s, l): ns = s + sq with its exact error by
        # Fast2Sum on (max, min) — s and sq are both >= +0, so the ordered
        # pair meets Fast2Sum's |a| >= |b| and the error is TwoSum's, bit for
        # bit (the C++ epilogue's), in 5 operations of dependency depth 3
        # instead of 6 of depth 5; s alternates between two registers
        for k in range(K):
            self.e("v_add_f64 %s, %s, -%s" % (P(SQ[k]), P(self.T(k)), P(Y[k])))
        for k in range(K):
            self.e("v_mul_f64 %s, %s, %s" % (P(SQ[k]), P(SQ[k]), P(SQ[k])))
        cur, other = HI, NS
        for k in range(K):
            self.e("v_add_f64 %s, %s, %s" % (P(other), P(cur), P(SQ[k])))
            self.e("v_max_f64 %s, %s, %s" % (P(BB), P(cur), P(SQ[k])))
            self.e("v_min_f64 %s, %s, %s" % (P(T2), P(cur), P(SQ[k])))
            self.e("v_add_f64 %s, %s, -%s" % (P(T1), P(other), P(BB)))
            self.e("v_add_f64 %s, %s, -%s" % (P(T1), P(T2), P(T1)))
            self.e("v_add_f64 %s, %s, %s" % (P(LO), P(LO), P(T1)))
            cur, other = other, cur
        if cur != HI:
            self.e("v_mov_b64_e32 %s, %s" % (P(HI), P(cur)))
        # a non-finite sum (inf/nan classes): the caller classifies it
        self.e("s_movk_i32 s%d, 0x207" % self.NXT)        # nan/inf classes
        self.e("v_cmp_class_f64_e64 vcc, %s, s%d" % (P(HI), self.NXT))
        self.e("s_and_b64 vcc, exec, vcc")
        self.e("s_cbranch_vccnz .Lend_%=")
        self.e("ds_write_b64 v%d, %s" % (A, P(HI)))
        self.e("ds_write_b64 v%d, %s offset:512" % (A, P(LO)))
        self.e("s_add_u32 s%d, s%d, 1" % (self.SJ, self.SJ))
        self.e("s_branch .Lnext_%=")

    def loop_end_hits(self):
        """END of a program in the typed loop core: the matches of bool(T)
        with the labels, counted per wave — f_eval's HITS_BOOL count, one
        ballot per case: ~(pred ^ %[lab_k]) & %[val_k] (the label and
        valid-case masks of this tile, k = 0..K-1) — added into lane j of
        %[hacc] (program j's running count in this tile group)."""
        CA, B = self.sp(self.CA), self.BASE
        if self.prefetch:
            # the next program's first window, loaded while the count is
            # formed (END waited for the leaf loads: no LDS wait follows
            # before .Lhave's, which then covers this load)
            self.e("s_add_u32 s%d, s%d, 1" % (self.SPF, self.SJ))
            self.e("s_cmp_lt_u32 s%d, %%[nmine]" % self.SPF)
            self.e("s_cbranch_scc0 .Lnopf_%=")
            self.load_first_window(self.SPF)
            self.label(".Lnopf_")
        for k in range(self.K):
            self.e("v_cmp_neq_f64_e64 %s, 0, %s" % (CA, self.p(self.T(k))))
            self.e("s_xnor_b64 %s, %s, %%[lab%d]" % (CA, CA, k))
            self.e("s_and_b64 %s, %s, %%[val%d]" % (CA, CA, k))
            self.e("s_bcnt1_i32_b64 s%d, %s" % (B + min(k, 1), CA))
            if k:
                self.e("s_add_u32 s%d, s%d, s%d" % (B, B, B + 1))
        self.e("v_readlane_b32 s%d, %%[hacc], s%d" % (self.NXT, self.SJ))
        self.e("s_nop 1")
        self.e("s_add_u32 s%d, s%d, s%d" % (self.NXT, self.NXT, B))
        # (one SGPR operand per VALU instruction: the lane select in M0,
        # free at END; .Lnext resets it)
        self.e("s_mov_b32 m0, s%d" % self.SJ)
        self.e("s_nop 0")
        self.e("v_writelane_b32 %%[hacc], s%d, m0" % self.NXT)
        self.e("s_add_u32 s%d, s%d, 1" % (self.SJ, self.SJ))
        self.e("s_branch .Lnext_%=")

    # ----------------------------------------------------------- build --
    def build(self):
        K, D, NV = self.K, self.D, self.NV
        P = self.p
        W, TC = self.WIN, self.TC
        # prologue: save M0, load the first window and the trig constants
        if self.m0lane:
            # the caller's M0 in lane 0 of VINF (unused by the exact cores):
            # s81 is then free, and s[80:81] a mask pair in the handlers
            self.e("s_nop 0")
            self.e("v_writelane_b32 v%d, m0, 0" % self.VINF)
        if self.salu:
            # the handlers' EXEC (SMASK): EXEC is the same at every handler's
            # entry (each restores it before its jump: check_exec); s101
            # (free: no window prefetch in the exact cores) the 0.855469
            # threshold of their first range compares
            assert not self.prefetch
            self.e("s_mov_b64 %s, exec" % self.sp(self.SMASK))
            self.e("s_mov_b32 s%d, 0x%x" % (self.SPF, GLIBC_T0855))
        else:
            self.e("s_mov_b32 s%d, m0" % self.SM0)
        if self.loop:
            self.e("s_mov_b32 s%d, %%[jio]" % self.SJ)
        if self.prefetch:
            self.e("s_mov_b32 s%d, -1" % self.SPF)
        self.prologue_base()
        if self.prio:
            self.e("s_setprio %d" % self.prio[0])
        if not self.loop:
            self.e("s_mov_b64 %s, %%[pc]" % self.sp(self.PTR))
        self.e("v_mov_b32_e32 v%d, 0" % self.VRED)
        if not self.exact:
            self.e("v_mov_b32_e32 v%d, 0" % self.VINF)
        self.e("s_cmp_eq_u32 %[probe], 0")
        self.e("s_cbranch_scc1 .Lrun_%=")
        self.e("s_branch .Lprobe_%=")
        self.label(".Lrun_")
        if not self.typed:
            self.e("s_load_dwordx16 s[%d:%d], %%[cst], 0x0" % (TC, TC + 15))
        if self.exact:
            self.e("s_load_dwordx16 s[%d:%d], %%[cst], 0x40"
                   % (self.TC2, self.TC2 + 15))
            if GLIBC2 and not GLIBC4:    # the cos-ordered __sincostab's offset
                assert not self.prefetch
                self.e("s_movk_i32 s%d, 0x%x" % (self.SPF, GLIBC_COSTAB))
        if self.loop:
            self.loop_next()
        else:
            self.e("s_load_dwordx16 s[%d:%d], %s, 0x0"
                   % (W, W + 15, self.sp(self.PTR)))
            self.e("s_mov_b32 m0, 0")
            self.e("s_waitcnt lgkmcnt(0)")
            self.e("s_nop 0")
            self.dispatch_head()
            self.dispatch_tail()
        # ---- handlers
        if self.align:                   # never reached by fall-through
            self.e(".p2align %d" % max(self.align, 6))
            self.label(".Lbase_")
        self.handler("END")
        self.e("s_waitcnt lgkmcnt(0)")       # a leaf load into T may be in flight
        if self.loop and self.typed:
            self.loop_end_hits()
        elif self.loop:
            self.loop_end()
        else:
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

        CA = self.sp(self.CA)
        self.handler("LDC")
        self.dispatch_head(2)
        self.e("s_waitcnt lgkmcnt(0)")
        for k in range(K):
            self.e("v_mov_b64_e32 %s, %s" % (P(self.T(k)), CA))
        self.dispatch_tail()
        # leaf loads into T: not waited for here — every handler that reads
        # or writes T waits (lgkmcnt(0)) first, so the LDS latency overlaps
        # the jump to it
        for v in range(NV):
            self.handler("LDV%d" % v)
            self.dispatch_head()
            self.ldx(self.T(0), v)
            self.dispatch_tail()
        # experiment (wrong values): pushes without their copies into the
        # stack slot — the most that renaming slots instead of copying
        # could save
        # could save; "dup_push_mov" (values unchanged): every
        # copy issued twice, the marginal cost of the copies
        push_mov = os.environ.get("GEN_ASM_EXPERIMENT") != "no_push_mov"
        if os.environ.get("GEN_ASM_EXPERIMENT") == "dup_push_mov":
            push_mov = 2
        for d in range(D):
            self.handler("PUSH%d" % d)
            self.dispatch_head()
            self.e("s_waitcnt lgkmcnt(0)")
            for k in list(range(K)) * int(push_mov):
                self.e("v_mov_b64_e32 %s, %s" % (P(self.R(d, k)),
                                                P(self.T(k))))
            self.dispatch_tail()
        for d in range(D):
            self.handler("PUSHC%d" % d)
            self.dispatch_head(2)
            self.e("s_waitcnt lgkmcnt(0)")
            for k in list(range(K)) * int(push_mov):
                self.e("v_mov_b64_e32 %s, %s" % (P(self.R(d, k)),
                                                P(self.T(k))))
            for k in range(K):
                self.e("v_mov_b64_e32 %s, %s" % (P(self.T(k)), CA))
            self.dispatch_tail()
        for d in range(D):
            for v in range(NV):
                self.handler("PUSHV%d_%d" % (d, v))
                self.dispatch_head()
                self.e("s_waitcnt lgkmcnt(0)")
                for k in list(range(K)) * int(push_mov):
                    self.e("v_mov_b64_e32 %s, %s" % (P(self.R(d, k)),
                                                    P(self.T(k))))
                self.ldx(self.T(0), v)
                self.dispatch_tail()
        for fam in self.fams:
            for d in range(D):
                self.handler("%s_S%d" % (fam, d))
                self.dispatch_head()
                self.e("s_waitcnt lgkmcnt(0)")
                self.binop_all(fam, [P(self.R(d, k)) for k in range(K)])
                self.dispatch_tail()
            shared = fam in ("div", "rdiv", "ndiv", "nrdiv")   # long bodies
            for v in range(NV):
                self.handler("%s_V%d" % (fam, v))
                self.ldx(self.O(0), v)
                self.dispatch_head()
                if shared:
                    self.e("s_branch .Lbody_%s_V_%%=" % fam)
                    continue
                self.e("s_waitcnt lgkmcnt(0)")
                self.binop_all(fam, [P(self.O(k)) for k in range(K)])
                self.dispatch_tail()
            if shared:
                self.label(".Lbody_%s_V_" % fam)
                self.e("s_waitcnt lgkmcnt(0)")
                self.binop_all(fam, [P(self.O(k)) for k in range(K)])
                self.dispatch_tail()
            self.handler("%s_C" % fam)
            self.dispatch_head(2)
            self.e("s_waitcnt lgkmcnt(0)")
            self.binop_all(fam, [CA] * K)
            self.dispatch_tail()
        self.handler("NEG")
        self.dispatch_head()
        self.e("s_waitcnt lgkmcnt(0)")
        for k in range(K):               # exact sign flip, as -x in Python
            self.e("v_xor_b32_e32 v%d, 0x80000000, v%d"
                   % (self.T(k) + 1, self.T(k) + 1))
        self.dispatch_tail()
        if self.typed:
            self.handler("NOT")
            self.dispatch_head()
            self.e("s_waitcnt lgkmcnt(0)")
            for k in range(K):             # (T == 0) ? 1.0 : 0.0
                self.e("v_cmp_eq_f64_e32 vcc, 0, %s" % P(self.T(k)))
                self.set_bool(k)
            self.dispatch_tail()
            for d in range(D - 1):         # if_then_else(stk[d], stk[d+1], T)
                self.handler("ITE%d" % d)
                self.dispatch_head()
                self.e("s_waitcnt lgkmcnt(0)")
                for k in range(K):
                    c, v, tk = self.R(d, k), self.R(d + 1, k), self.T(k)
                    self.e("v_cmp_neq_f64_e32 vcc, 0, %s" % P(c))
                    self.e("v_cndmask_b32_e32 v%d, v%d, v%d, vcc" % (tk, tk, v))
                    self.e("v_cndmask_b32_e32 v%d, v%d, v%d, vcc"
                           % (tk + 1, tk + 1, v + 1))
                self.dispatch_tail()
        for want in (() if self.typed else ("sin", "cos")):
            self.handler(want.upper())
            self.dispatch_head()
            self.e("s_waitcnt lgkmcnt(0)")
            if self.exact:                 # glibc's sin/cos, chains interleaved
                if not GLIBC2:             # (glibc_ops2 keeps VRED itself)
                    self.vred_update()     # (GEN_ASM_EXACT_SEQ=1: in turn)
                n0 = len(self.lines)
                self.sincos(want, mixed=os.environ.get("GEN_ASM_EXACT_SEQ") == "1")
                if self.prio and GLIBC2:   # (the bodies drop it after their gathers)
                    self.e("s_setprio %d" % self.prio[0])
                elif self.prio:
                    if self.prio_late:
                        self.late_prio(n0)
                    else:
                        self.lines.insert(n0, "s_setprio %d" % self.prio[1])
                    self.e("s_setprio %d" % self.prio[0])
                self.dispatch_tail()
                self.flush_ool()
                continue
            if self.prio and not self.prio_late:   # the trig body at the other priority
                self.e("s_setprio %d" % self.prio[1])
            self.trig_prefix(want)
            n0 = len(self.lines)
            self.sincos(want)
            self.late_prio(n0)
            if self.prio:
                self.e("s_setprio %d" % self.prio[0])
            self.dispatch_tail()
            self.label(".Lmix_%s_" % want)
            self.vred_update()
            n0 = len(self.lines)
            self.sincos(want, mixed=True)
            self.late_prio(n0)
            if self.prio:
                self.e("s_setprio %d" % self.prio[0])
            self.dispatch_tail()
        # ---- probe: write the handler offset table
        self.label(".Lprobe_")
        self.probe_stores(self.POOL0, self.POOL0 + 1)
        self.label(".Lend_")
        if self.prefetch:
            self.e("s_waitcnt lgkmcnt(0)")     # no window load past the core
        if self.prio:
            self.e("s_setprio 0")
        if self.loop:
            self.e("s_mov_b32 %%[jio], s%d" % self.SJ)
        # results: T and the running max of |x|.hi stay where they are (the
        # asm outputs are bound to those VGPRs: no copies, and no registers
        # of the compiler's own held for them across the core)
        if self.m0lane:
            self.e("v_readlane_b32 s%d, v%d, 0" % (self.SM0, self.VINF))
            self.e("s_nop 0")
            self.e("s_mov_b32 m0, s%d" % self.SM0)
        else:
            self.e("s_mov_b32 m0, s%d" % self.SM0)
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
        for f, fam in enumerate(self.fams):
            assert ids["%s_S0" % fam] == base_bin + f * stride
            assert ids["%s_V0" % fam] == base_bin + f * stride + D
            assert ids["%s_C" % fam] == base_bin + f * stride + D + NV
        assert ids["PUSHV%d_%d" % (D - 1, NV - 1)] == \
            base_pushv + (D - 1) * NV + NV - 1
        out = {"H_END": ids["END"], "H_RELOAD": ids["RELOAD"],
               "H_LDC": ids["LDC"], "H_LDV0": base_ldv,
               "H_PUSH0": base_push, "H_PUSHC0": base_pushc,
               "H_PUSHV0": base_pushv, "H_BIN0": base_bin,
               "H_FAM_STRIDE": stride, "H_NEG": ids["NEG"],
               "H_SIN": ids.get("SIN", -1), "H_COS": ids.get("COS", -1),
               "H_COUNT": len(names), "WINDOW": WINDOW,
               "SGPR_BASE": self.BASE,
               "LIM_HI": LIM_HI, "FAST_HI": FAST_HI}
        if self.typed:
            assert ids["ITE%d" % (D - 2)] == ids["ITE0"] + D - 2
            out.update(H_NOT=ids["NOT"], H_ITE0=ids["ITE0"],
                       N_FAMS=len(self.fams))
        return out


def check_exec(lines, saved):
    """Every path through every handler that changes EXEC restores it from
    `saved` (the handler's EXEC, an SGPR pair) before its jump: an EXEC left
    partial would run the next handlers — and the C++ around the core — on
    a subset of the lanes (or none: a uniform loop there never ends).
    Raises AssertionError with the path's last label otherwise."""
    lab = {}
    for i, l in enumerate(lines):
        if l.endswith(":") and not l.startswith("s_") and not l.startswith("v_"):
            lab[l[:-1]] = i
    seen = set()
    starts = [i + 1 for i, l in enumerate(lines) if l.startswith(".Lh_")]
    for st in starts:
        stack = [(st, True)]
        while stack:
            i, clean = stack.pop()
            while i < len(lines):
                if (i, clean) in seen:
                    break
                seen.add((i, clean))
                l = lines[i]
                if l.startswith(".Lh_"):
                    break                       # (falls into the next handler)
                m = re.match(r"s_\w+ exec, (.*)$", l)
                if m:
                    clean = l.startswith("s_mov_b64") and m.group(1).strip() == saved
                if l.startswith("v_cmpx"):              # (writes EXEC too)
                    clean = False
                if l.startswith("s_setpc_b64"):
                    assert clean, "EXEC not restored before %r (line %d)" % (l, i)
                    break
                m = re.match(r"s_(cbranch_\w+|branch) (\S+)$", l)
                if m:
                    assert m.group(2) in lab, m.group(2)
                    if m.group(1) == "branch":
                        i = lab[m.group(2)]
                        continue
                    stack.append((lab[m.group(2)], clean))
                i += 1


def trig_data():
    """Table + constants of the table-driven sin/cos (trig_table.json)."""
    import json
    with open(os.path.join(HERE, "trig_table.json")) as fh:
        return json.load(fh)


def trig_const_block():
    """Doubles of the C++ gp_trig (kTrigConst, 16) — INV, S1, 0, -S2, LIM,
    TINY, FAST, Ps0, Ps1, Ps2, Pc1, Pc2, C1, C2, C3, MAGIC — followed by
    the asm core's SGPR block (kAsmConst, 8; SGPR_CONSTS order).  S1 + S2
    serve the fast reduction below FAST = 2^14 (FAST_HI), C1 + C2 + C3 the
    long one up to LIM = 2^40 (LIM_HI)."""
    d = trig_data()
    ps, pc, cc = d["Ps"], d["Pc"], d["C"]
    assert float.fromhex(pc[0]) == -0.5      # an inline constant in the core
    ns2 = (-float.fromhex(d["S2"])).hex()
    cpp = [d["INV"], d["S1"], "0x0p+0", ns2, "0x1p+40", "0x1p-26",
           "0x1p+%d" % FAST_EXP, ps[0], ps[1], ps[2], pc[1], pc[2], cc[0], cc[1], cc[2],
           MAGIC]

    val = {"INV": d["INV"], "S1": d["S1"], "FAST": "0x1p+%d" % FAST_EXP, "NS2": ns2,
           "Ps0": ps[0], "Ps1": ps[1], "Pc1": pc[1], "C1": cc[0]}
    core = [val[n] for n in SGPR_CONSTS]
    # LDS words after the table: (Ps2, Pc2) (the cores take them as VGPR
    # operands instead), (C2, C3)
    lds_tail = [ps[2], pc[2], cc[1], cc[2]]
    return cpp, core, lds_tail


def emit(K, D, NV, suffix="", out_dir=HERE, trig_group=0):
    """Writes ``gp_asm_core<suffix>.inc`` (macros ``GP_ASM_CORE<SUFFIX>``
    ...) and ``gp_asm_layout<suffix>.h`` (namespace ``asmcore<suffix>``).
    The library carries two fp64 cores: D = 5 (the fast one) and a deep one
    for programs that need more operand-stack slots."""
    exact = suffix in ("_exact", "_exact_deep")    # glibc sin/cos (redo pass)
    typed = suffix == "_typed"
    # the D = 5 core runs the wave's program loop itself (Gen.loop); its
    # registers start at GEN_ASM_TB0 (the caller keeps fewer registers live
    # across a looping core).  The typed core always loops.
    loop = typed or (suffix in ("", "_exact") and
                     os.environ.get("GEN_ASM_LOOP", "1") == "1")
    tb0 = int(os.environ.get("GEN_ASM_TB0", "32")) if suffix == "" else 32
    # trig_group: sin/cos chains interleaved that many at a time (0: all K);
    # K = 4 cores run them one by one (their temporaries set the VGPRs)
    g = Gen(K, D, NV, TB0=tb0, exact=exact, loop=loop, typed=typed,
            trig_group=trig_group).build()
    # experiment knob: reserve more VGPRs (clobbered, unused) to price the
    # occupancy a register-hungrier core would have
    g.vmax += int(os.environ.get("GEN_ASM_PAD_VGPRS", "0")) if not suffix else 0
    S = suffix.upper()
    lay = g.layout()
    body = g.lines
    if exact:
        check_exec(body, g.sp(g.SMASK))
    inc = os.path.join(out_dir, "gp_asm_core%s.inc" % suffix)
    with open(inc, "w") as fh:
        fh.write("// GENERATED by gen_asm.py (K=%d, D=%d, NV=%d) — do not edit\n"
                 % (K, D, NV))
        if suffix in ("", "_exact"):
            fh.write("#define GP_ASM_LOOP%s %d\n" % (suffix.upper(),
                                                     1 if g.loop else 0))
        fh.write("#define GP_ASM_CORE%s \\\n" % S)
        for l in body:
            fh.write('  "%s\\n" \\\n' % l)
        fh.write('  ""\n')
        outs = set(range(g.TB0, g.TB0 + 2 * K)) | {g.VRED}
        if not exact:
            outs.add(g.VINF)
        clob = ['"v%d"' % r for r in range(g.TB0, g.vmax) if r not in outs]
        clob += ['"s%d"' % r for r in range(g.SB, g.SMAX + 1)]
        clob += ['"vcc"', '"scc"', '"memory"']
        fh.write("#define GP_ASM_CLOBBERS%s %s\n" % (S, ", ".join(clob)))
        fh.write("#define GP_ASM_T_OUTPUTS%s %s\n" % (S, ", ".join(
            '[T%d] "=&{v[%d:%d]}"(T[%d])' % (k, g.T(k), g.T(k) + 1, k)
            for k in range(K))))
        fh.write('#define GP_ASM_VRED_OUTPUT%s [vred] "=&{v%d}"(vred)\n'
                 % (S, g.VRED))
        if not exact:
            fh.write('#define GP_ASM_VINF_OUTPUT%s [vinf] "=&{v%d}"(vinf)\n'
                     % (S, g.VINF))
        else:        # the VGPR constants (gpeval.hip namespace glibc)
            ins = []
            for n in GLIBC_VGPR:
                if GLIBC3 and n.startswith("HP1_"):    # (glibc_seq3: SGPRs)
                    continue
                if n.startswith("HP1_"):
                    sh = 32 if n.endswith("HI") else 0
                    val = ("(uint32_t)(__builtin_bit_cast(uint64_t, glibc::HP1)"
                           " >> %d)" % sh)
                else:
                    val = "glibc::%s" % n
                ins.append('[g_%s] "v"(%s)' % (n.lower(), val))
            fh.write("#define GP_ASM_GLIBC_INPUTS%s %s\n" % (S, ", ".join(ins)))
    hdr = os.path.join(out_dir, "gp_asm_layout%s.h" % suffix)
    cpp, core, lds_tail = trig_const_block()
    with open(hdr, "w") as fh:
        fh.write("// GENERATED by gen_asm.py — handler id layout\n")
        fh.write("namespace asmcore%s {\n" % suffix)
        fh.write("constexpr int K = %d, D = %d, NV = %d;\n" % (K, D, NV))
        fh.write("constexpr int VGPRS = %d;  // highest VGPR used + 1\n"
                 % g.vmax)
        fh.write("constexpr bool LOOP = %s;  // the core runs the program loop\n"
                 % ("true" if g.loop else "false"))
        if exact:
            fh.write("constexpr int GLIBC_LDS_BYTES = %d;  // tables + constants\n"
                     % GLIBC_LDS_BYTES)
            fh.write("// __sincostab's LDS image: 1 = three arrays (sn, ssn), (cs, ccs),\n"
                     "// (-sn, -ssn) GLIBC_SPLIT_S bytes apart (glibc_seq4); 0 = the table,\n"
                     "// then (after __branred's data) its cos-ordered copy\n")
            fh.write("constexpr int GLIBC_TAB_SPLIT = %d, GLIBC_SPLIT_S = %d;\n"
                     % (1 if GLIBC4 else 0, GLIBC_SPLIT_S))
            fh.write("// the caller's M0 kept in lane 0 of VINF (1) or in s81 (0)\n")
            fh.write("constexpr int M0_LANE = %d;\n" % (1 if g.m0lane else 0))
            fh.write("constexpr int GLIBC_BRANRED_OFF = %d;  // SPLIT, BBIG1, BMP2, pad, toverp\n"
                     % GLIBC_BRANRED_BYTES)
            fh.write("constexpr uint32_t BRANRED_HI = 0x%x;\n" % BRANRED_HI)
            fh.write("// vred at or past this (inf, nan): the C++ exact pass\n")
            fh.write("constexpr uint32_t EXACT_REDO_HI = 0x7ff00000;\n")
            fh.write("// LDS after __sincostab: %s, then toverp[75], one pad\n"
                     % ", ".join(GLIBC_BRANRED_CONSTS))
            fh.write("// d_cst doubles 0..15 (the SGPR blocks): %s\n"
                     % ", ".join(GLIBC_SGPR))
        for k, v in lay.items():
            fh.write("constexpr int %s = %d;\n" % (k, v))
        fh.write("constexpr double kTrigConst[16] = {\n    %s};\n"
                 % ",\n    ".join(cpp))
        fh.write("constexpr double kAsmConst[8] = {\n    %s};\n"
                 % ",\n    ".join(core))
        fh.write("constexpr int kTrigEntries = %d;  // sin(j pi/256), j < %d\n"
                 % (TAB_ENTRIES, TAB_ENTRIES))
        fh.write("// the LDS image of the table: 0 (hi, lo) entries, 1 hi parts "
                 "then lo parts\n")
        fh.write("constexpr int SPLIT_TAB = %d;\n" % (1 if SPLIT_TAB else 0))
        fh.write("constexpr double kTrigTable[%d * 2] = {\n    %s};\n"
                 % (TAB_ENTRIES, ",\n    ".join(
                     v for row in trig_data()["table"] for v in row)))
        fh.write("constexpr double kTrigLdsTail[4] = {\n    %s};\n"
                 % ",\n    ".join(lds_tail))
        # the cores' VGPR-pair operands %[mg], %[ps2], %[pc2]
        fh.write("constexpr double kAsmMagic = %s, kAsmPs2 = %s, kAsmPc2 = %s;\n"
                 % (MAGIC, lds_tail[0], lds_tail[1]))

        if not suffix:        # glibc_sin/cos tables (gen_trig_table.py)
            d = trig_data()
            fh.write("constexpr double kGlibcSincostab[440] = {\n    %s};\n"
                     % ",\n    ".join(d["glibc_sincostab"]))
            fh.write("constexpr double kGlibcToverp[75] = {\n    %s};\n"
                     % ",\n    ".join("%d.0" % v for v in d["glibc_toverp"]))
        fh.write("}  // namespace asmcore%s\n" % suffix)
    return inc, hdr, lay, g.vmax


if __name__ == "__main__":
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    D = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    NV = int(sys.argv[3]) if len(sys.argv) > 3 else 32
    SUF = sys.argv[4] if len(sys.argv) > 4 else ""
    TG = int(sys.argv[5]) if len(sys.argv) > 5 else 0
    print(emit(K, D, NV, SUF, trig_group=TG))
