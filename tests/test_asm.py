"""The hand-scheduled asm interpreter core, checked on the CPU (no GPU).

1. The device code object is disassembled; the handler table that the probe
   kernel would write is read back from its immediates, and every entry must
   land on an instruction boundary of ``f_eval_asm`` that starts the expected
   handler (a wrong jump target would execute garbage on the GPU).
2. Golden programs are translated by the library's own translator
   (``gpe_debug_translate``) with that table and the resulting threaded code
   is executed by a Python model of the handlers; it must reproduce the
   bytecode mirror (tests/bytecode_ref.py) bit for bit.
"""
import math
import os
import re
import subprocess
import sys

import numpy as np
import pytest

import bytecode_ref as ref
from conftest import REPO, load_golden
from deap_amd import _lib, build, configs, datasets, gp
from deap_amd.flatten import Flattener

LLVM = "/opt/rocm/lib/llvm/bin"


# the two fp64 cores: D = 5 and deep (gp_asm_layout<suffix>.h), with the
# mangled-name keys of their probe and evaluation kernels
CORES = {"": ("11f_probe_asmE", "f_eval_asmILb0ELb0ELb0E"),
         "_deep": ("16f_probe_asm_deepE", "f_eval_asmILb0ELb1ELb0E"),
         "_typed": ("17f_probe_asm_typedE", "16f_eval_asm_typedE")}


def _layout(core=""):
    path = os.path.join(REPO, "deap_amd", "csrc", "gp_asm_layout%s.h" % core)
    vals = dict(re.findall(r"constexpr int (\w+) = (\d+);",
                           open(path).read()))
    k, d, nv = re.search(r"constexpr int K = (\d+), D = (\d+), NV = (\d+);",
                         open(path).read()).groups()
    out = {k_: int(v) for k_, v in vals.items()}
    out.update(K=int(k), D=int(d), NV=int(nv))
    return out


@pytest.fixture(scope="module")
def disasm(tmp_path_factory):
    # the gfx950 code object of the built library itself (its offload
    # bundle), not a second compile
    build.build()
    tmp = tmp_path_factory.mktemp("dev")
    lib = os.path.join(REPO, "deap_amd", "libgpeval.so")
    subprocess.run(["objcopy", "--dump-section", ".hip_fatbin=%s" % (tmp / "fat.bin"),
                    lib, str(tmp / "lib.stripped")], check=True, capture_output=True)
    subprocess.run([LLVM + "/clang-offload-bundler", "--unbundle", "--type=o",
                    "--input=%s" % (tmp / "fat.bin"), "--output=%s" % (tmp / "g.co"),
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950"],
                   check=True, capture_output=True)
    text = subprocess.run([LLVM + "/llvm-objdump", "-d", "--no-show-raw-insn",
                           str(tmp / "g.co")], capture_output=True, text=True,
                          check=True).stdout
    funcs = {}
    cur = None
    for line in text.splitlines():
        m = re.match(r"^([0-9a-f]+) <(.+)>:$", line)
        if m:
            cur = m.group(2)
            funcs[cur] = []
            continue
        m = re.search(r"//\s*([0-9A-F]{12}):", line)
        if cur and m:
            funcs[cur].append((int(m.group(1), 16),
                               line.split("//")[0].strip()))
    return funcs


def _func(funcs, key):
    return [v for k, v in funcs.items() if key in k][0]


def _base(insts, core=""):
    b = _layout(core)["SGPR_BASE"]
    want = "s_getpc_b64 s[%d:%d]" % (b, b + 1)
    for i, (addr, txt) in enumerate(insts):
        if txt.startswith(want):
            return addr + 4
    raise AssertionError("no " + want)


def probe_table(funcs, core=""):
    insts = _func(funcs, CORES[core][0])
    table = {}
    last_mov = None
    base = 0                      # the store address moves on past 4 KiB
    for addr, txt in insts:
        if re.match(r"v_add_u32_e32 v\d+, 0x800, v\d+$", txt):
            base += 0x800
            continue
        m = re.match(r"v_mov_b32_e32 v\d+, (0x[0-9a-f]+|\d+)$", txt)
        if m:
            last_mov = int(m.group(1), 0)
            continue
        m = re.match(r"global_store_dword v\d+, v\d+, s\[\d+:\d+\]"
                     r"(?: offset:(\d+))?$", txt)
        if m and last_mov is not None:
            table[(base + int(m.group(1) or 0)) // 4] = last_mov
            last_mov = None
    n = max(table) + 1
    assert sorted(table) == list(range(n))
    return np.array([table[i] for i in range(n)], dtype=np.uint32)


@pytest.mark.parametrize("core", sorted(CORES))
def test_handler_table_targets_are_handler_entries(disasm, core):
    lay = _layout(core)
    table = probe_table(disasm, core)
    assert len(table) == lay["H_COUNT"]
    insts = _func(disasm, CORES[core][1])
    base = _base(insts, core)
    at = {addr: txt for addr, txt in insts}
    K, D, NV = lay["K"], lay["D"], lay["NV"]
    for hid, off in enumerate(table):
        txt = at.get(base + int(off))
        assert txt is not None, "handler %d: not an instruction boundary" % hid
        if hid == lay["H_END"]:
            # waits for a leaf load still in flight, then leaves the core
            assert txt.startswith("s_waitcnt lgkmcnt(0)"), txt
        elif hid == lay["H_RELOAD"]:
            assert txt.startswith("s_add_u32"), txt
        else:
            bin0, st = lay["H_BIN0"], lay["H_FAM_STRIDE"]
            r = (hid - bin0) % st
            n_fams = lay.get("N_FAMS", 8)
            if bin0 <= hid < bin0 + n_fams * st and D <= r < D + NV:
                assert txt.startswith("ds_read_b64"), (hid, txt)
            else:
                assert txt.startswith("s_movrels_b32"), (hid, txt)
    # the probe and the evaluator assemble the same core: identical layout
    pinsts = _func(disasm, CORES[core][0])
    pbase = _base(pinsts, core)
    pat = {addr - pbase: txt for addr, txt in pinsts}
    eat = {addr - base: txt for addr, txt in insts}
    mnem = lambda t: t.split()[0] if t else t      # operands of compiler-
    for off in table:                              # assigned inputs differ
        assert mnem(pat.get(int(off))) == mnem(eat.get(int(off)))


# ------------------------------------------------- threaded-code model --
def _decode(lay, hid):
    K, D, NV = lay["K"], lay["D"], lay["NV"]
    fams = ["add", "sub", "rsub", "mul", "div", "rdiv", "ndiv", "nrdiv"]
    if hid == lay["H_END"]:
        return ("END",)
    if hid == lay["H_RELOAD"]:
        return ("RELOAD",)
    if hid == lay["H_LDC"]:
        return ("LDC",)
    if lay["H_LDV0"] <= hid < lay["H_LDV0"] + NV:
        return ("LDV", hid - lay["H_LDV0"])
    if lay["H_PUSH0"] <= hid < lay["H_PUSH0"] + D:
        return ("PUSH", hid - lay["H_PUSH0"])
    if lay["H_PUSHC0"] <= hid < lay["H_PUSHC0"] + D:
        return ("PUSHC", hid - lay["H_PUSHC0"])
    if lay["H_PUSHV0"] <= hid < lay["H_PUSHV0"] + D * NV:
        r = hid - lay["H_PUSHV0"]
        return ("PUSHV", r // NV, r % NV)
    b = hid - lay["H_BIN0"]
    st = lay["H_FAM_STRIDE"]
    if 0 <= b < 8 * st:
        fam, r = fams[b // st], b % st
        if r < D:
            return ("BIN", fam, "S", r)
        if r < D + NV:
            return ("BIN", fam, "V", r - D)
        return ("BIN", fam, "C")
    return {lay["H_NEG"]: ("NEG",), lay["H_SIN"]: ("SIN",),
            lay["H_COS"]: ("COS",)}[hid]


def run_threaded(words, start, inv, lay, X):
    n = X.shape[1]
    T = np.zeros(n)
    R = {}
    verr = np.zeros(n, dtype=bool)
    pc = start

    def const():
        return ref._f64(words[pc], words[pc + 1])
    while True:
        h = _decode(lay, inv[int(words[pc])])
        pc += 1
        if h[0] == "END":
            return T, verr
        if h[0] == "RELOAD":                 # next 16-word window
            pc = ((pc - 1) // lay["WINDOW"] + 1) * lay["WINDOW"]
            continue
        if h[0] == "LDC":
            T = np.full(n, const()); pc += 2
        elif h[0] == "LDV":
            T = X[h[1]].copy()
        elif h[0] == "PUSH":
            R[h[1]] = T
        elif h[0] == "PUSHC":
            R[h[1]] = T; T = np.full(n, const()); pc += 2
        elif h[0] == "PUSHV":
            R[h[1]] = T; T = X[h[2]].copy()
        elif h[0] == "BIN":
            if h[2] == "S":
                a = R[h[3]]
            elif h[2] == "V":
                a = X[h[3]]
            else:
                a = const(); pc += 2
            T = ref._fbin(h[1], a, T)
        elif h[0] == "NEG":
            T = -T
        else:
            verr |= np.isinf(T)
            fn = math.sin if h[0] == "SIN" else math.cos
            T = np.array([fn(v) if math.isfinite(v) else math.nan
                          for v in T.tolist()])


def _deep_trees():
    """Taller config-4 trees: every one of a seeded pool that needs more
    than 5 operand-stack slots, plus 20 that do not."""
    pset = configs.pset_for("symreg10")
    pool = configs.population(pset, "half", 600, 11, 9, 12)
    depth = Flattener(pset).flatten(pool).depth
    keep = [t for t, d in zip(pool, depth) if d > 5][:40]
    keep += [t for t, d in zip(pool, depth) if d <= 5][:20]
    return {"pset": "symreg10", "trees": [str(t) for t in keep]}


@pytest.mark.parametrize("core", ["", "_deep"])    # (the typed core: STGP
@pytest.mark.parametrize("name", ["c1_symbreg", "c1_edge", "c4_symreg10",   # goldens
                                  "deep_trees"])                           # on the GPU)
def test_translation_matches_bytecode(disasm, name, core):
    lay = _layout(core)
    table = probe_table(disasm, core)
    inv = {int(off): hid for hid, off in enumerate(table)}
    g = _deep_trees() if name == "deep_trees" else load_golden(name)
    pset = configs.pset_for(g["pset"])
    trees = [gp.PrimitiveTree.from_string(s, pset) for s in g["trees"]]
    batch = Flattener(pset).flatten(trees)
    if g["pset"] == "symbreg":
        X, _ = datasets.symbreg_points()
    else:
        X, _ = datasets.symreg10_cases(256, 3)
    words, starts = _lib.debug_translate(batch, X.shape[0], table)
    n_asm = 0
    for i in range(len(trees)):
        code = batch.code[batch.offsets[i]:batch.offsets[i + 1]]
        if starts[i] < 0:
            assert batch.depth[i] > lay["D"] or batch.err[i] != 0
            continue
        n_asm += 1
        a, va = run_threaded(words, int(starts[i]), inv, lay, X)
        b, vb = ref.run_f(code, X)
        assert np.array_equal(a.view(np.uint64), b.view(np.uint64)) or \
            np.array_equal(np.isnan(a), np.isnan(b)) and \
            np.array_equal(a[~np.isnan(a)], b[~np.isnan(b)]), g["trees"][i]
        assert np.array_equal(va, vb)
    if name == "deep_trees":
        deeper = int((batch.depth > _layout()["D"]).sum())
        assert deeper >= 10
        assert n_asm == len(trees) - (deeper if core == "" else 0)
    elif name != "c1_edge":
        assert n_asm >= 0.9 * len(trees)


def test_fp32_argument_key_orders_the_classes():
    """gen_asm32.py's sin/cos argument key (2|x|.bits - 2 LIM mod 2^32, min
    over the arguments): finite >= 2^30 < +-inf < nan < finite < 2^30, so
    the kernel re-runs on key < RED_INF and raises ValueError on == RED_INF
    whichever order the arguments came in."""
    import struct
    import sys
    sys.path.insert(0, os.path.join(REPO, "deap_amd", "csrc"))
    import gen_asm32 as g

    def key(v):
        b = struct.unpack("<I", struct.pack("<f", v))[0]
        return ((b << 1) + g.RED_BIAS) & 0xffffffff
    big = [2.0 ** 30, -3e38, 1e10, -(2.0 ** 30)]
    small = [0.0, -0.0, 1.0, -5e8, 1e-45, 1073741760.0]
    inf = [math.inf, -math.inf]
    for b in big:
        assert key(b) < g.RED_INF
        for o in small + inf + [math.nan]:
            assert min(key(b), key(o)) < g.RED_INF
    for i in inf:
        assert key(i) == g.RED_INF
        for o in small + [math.nan]:
            assert min(key(i), key(o)) == g.RED_INF
    assert key(math.nan) > g.RED_INF
    for s_ in small:
        assert key(s_) > key(math.nan)
    rb = struct.unpack("<I", struct.pack("<f", dict(g.CONSTS)["RED"]))[0]
    assert rb == g.RED_BIAS


def test_one_copy_of_each_core_per_kernel(disasm):
    """Program words are absolute handler addresses of the kernel's own copy
    of its core (probed once through its one call site): a kernel holding
    two copies would jump from one into the other."""
    # the exact core keeps its handler base at a lower SGPR block (it needs
    # 16 more SGPRs for glibc's constants)
    want = tuple("s_getpc_b64 s[%d:%d]" % (b, b + 1) for b in
                 {_layout(s)["SGPR_BASE"] for s in ("", "_deep", "_exact", "_typed")})
    seen = 0
    for name, insts in disasm.items():
        n = sum(1 for _, txt in insts if txt.startswith(want))
        if "f_eval_asm" in name or "asm_values" in name or "f_probe_asm" in name:
            assert n == 1, (name, n)
            seen += 1
    assert seen >= 13


def test_product_cores_are_the_generators_defaults(tmp_path, monkeypatch):
    """The built cores are the generators' defaults: regenerated here with
    no GEN_ASM_* switch they are byte-identical, and a measurement switch in
    the caller's environment (scripts/build_variant.sh's experiments) does
    not reach the product build."""
    monkeypatch.setenv("GEN_ASM_EXPERIMENT", "dup_push_mov")
    build.generate()
    env = build._gen_env()
    assert "GEN_ASM_EXPERIMENT" not in env
    cmd = ("import sys; sys.path.insert(0, %r); import gen_asm, gen_asm32\n"
           "for a in %r: gen_asm.emit(int(a[0]), int(a[1]), int(a[2]), a[3], "
           "out_dir=%r, trig_group=int(a[4]) if len(a) > 4 else 0)\n"
           "for a in %r: gen_asm32.emit(int(a[0]), int(a[1]), int(a[2]), a[3], "
           "out_dir=%r)\n"
           % (os.path.join(REPO, "deap_amd", "csrc"),
              [list(build.ASM_VARIANT), build._deep(build.ASM_K2),
               list(build.ASM_K2) + ["_exact"], list(build.ASM_TYPED),
               build._deep(build.ASM_K2)[:3] + ["_exact_deep"]], str(tmp_path),
              [list(build.ASM32_VARIANT) + [""], build._deep(build.ASM32_VARIANT)],
              str(tmp_path)))
    subprocess.run([sys.executable, "-c", cmd], check=True, env=env,
                   stdout=subprocess.DEVNULL)
    for path in build.ASM_OUT + build.ASM32_OUT:
        fresh = tmp_path / os.path.basename(path)
        assert fresh.read_bytes() == open(path, "rb").read(), path


def test_exec_restore_checker():
    """gen_asm.check_exec (run on every exact core at generation): a handler
    path that jumps on with a partial EXEC is refused; restored paths pass."""
    sys.path.insert(0, os.path.join(REPO, "deap_amd", "csrc"))
    import gen_asm
    ok = [".Lh_A_%=:", "s_mov_b64 exec, s[1:2]", "s_cbranch_execz .La_%=",
          "v_mov_b32_e32 v0, 0", ".La_%=:", "s_mov_b64 exec, s[8:9]",
          "s_setpc_b64 s[4:5]"]
    gen_asm.check_exec(ok, "s[8:9]")
    bad = [".Lh_A_%=:", "s_or_b64 exec, s[1:2], s[3:4]", "s_cbranch_execz .La_%=",
           "v_mov_b32_e32 v0, 0", "s_mov_b64 exec, s[8:9]", ".La_%=:",
           "s_setpc_b64 s[4:5]"]
    with pytest.raises(AssertionError):
        gen_asm.check_exec(bad, "s[8:9]")
