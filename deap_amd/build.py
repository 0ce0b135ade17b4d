"""Build ``libgpeval.so`` in-tree for gfx950 (``python -m deap_amd.build``).

hipcc cross-compiles here without a GPU; the .so travels to the GPU box with
the repository snapshot.  ``-ffp-contract=off`` keeps every fp64 operation a
separately rounded IEEE operation, as in CPython.
"""
import os
import subprocess
import sys
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
SRC = os.path.join(HERE, "csrc", "gpeval.hip")
OUT = os.path.join(HERE, "libgpeval.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-ffp-contract=off", "-fPIC",
         "-shared", "-std=c++17", "-Wall", "-Wno-unused-function"]


GEN = os.path.join(HERE, "csrc", "gen_asm.py")
GEN32 = os.path.join(HERE, "csrc", "gen_asm32.py")
# the D = 5 core (the hot one): K cases per lane (GPE_ASM_K; 4 halves the
# dispatches per case but measured 1.3 % slower on C4: its sin/cos chains run
# one by one to stay at 4 waves per SIMD), stack slots, vars, sin/cos chains
# interleaved (0: all K)
ASM_K = os.environ.get("GPE_ASM_K", "2")
ASM_VARIANT = (ASM_K, "5", "32", "", "1" if int(ASM_K) > 2 else "0")
ASM_K2 = ("2", "5", "32")                # the deep and exact cores: K = 2
ASM32_VARIANT = ("4", "5", "32")         # the fp32 core: same layout, K = 4
ASM_DEEP_D = "12"                        # stack slots of the deep cores
ASM_TYPED = ("2", "5", "64", "_typed")   # the typed (STGP, HITS_BOOL) core
ASM_OUT = [os.path.join(HERE, "csrc", "gp_asm_core.inc"),
           os.path.join(HERE, "csrc", "gp_asm_layout.h"),
           os.path.join(HERE, "csrc", "gp_asm_core_deep.inc"),
           os.path.join(HERE, "csrc", "gp_asm_layout_deep.h"),
           os.path.join(HERE, "csrc", "gp_asm_core_exact.inc"),
           os.path.join(HERE, "csrc", "gp_asm_layout_exact.h"),
           os.path.join(HERE, "csrc", "gp_asm_core_typed.inc"),
           os.path.join(HERE, "csrc", "gp_asm_layout_typed.h"),
           os.path.join(HERE, "csrc", "gp_asm_core_exact_deep.inc"),
           os.path.join(HERE, "csrc", "gp_asm_layout_exact_deep.h")]
ASM32_OUT = [os.path.join(HERE, "csrc", "gp_asm_core32.inc"),
             os.path.join(HERE, "csrc", "gp_asm_core32_deep.inc")]


def _stale(outs, gens):
    newest = max(os.path.getmtime(g) for g in gens)
    return not all(os.path.exists(o) and os.path.getmtime(o) >= newest
                   for o in outs)


def _deep(variant):
    return [variant[0], ASM_DEEP_D, variant[2], "_deep"]


def _stamp():
    """The generator settings the cores were last generated with."""
    return os.path.join(HERE, "csrc", ".gp_asm_variant")


def _gen_env():
    """The generators' environment without their GEN_ASM_* experiment
    switches: the product cores are the generators' defaults whatever the
    caller's shell holds (experimental cores are built by
    scripts/build_variant.sh, into separate libraries)."""
    return {k: v for k, v in os.environ.items() if not k.startswith("GEN_ASM")}


def generate():
    """Regenerate the asm interpreter cores (gen_asm.py, gen_asm32.py: the
    D = 5 cores and the deep ones) if stale."""
    want = " ".join(ASM_VARIANT)
    try:
        with open(_stamp()) as fh:
            have = fh.read()
    except OSError:
        have = None
    if _stale(ASM_OUT, [GEN]) or have != want:
        # the D = 5 core, the deep one and the exact one (glibc sin/cos)
        for args in (list(ASM_VARIANT), _deep(ASM_K2),
                     list(ASM_K2) + ["_exact"], list(ASM_TYPED),
                     _deep(ASM_K2)[:3] + ["_exact_deep"]):
            subprocess.run([sys.executable, GEN] + args, check=True,
                           stdout=subprocess.DEVNULL, env=_gen_env())
        with open(_stamp(), "w") as fh:
            fh.write(want)
    if _stale(ASM32_OUT, [GEN, GEN32]):
        for args in (list(ASM32_VARIANT), _deep(ASM32_VARIANT)):
            subprocess.run([sys.executable, GEN32] + args, check=True,
                           stdout=subprocess.DEVNULL, env=_gen_env())


# the headers of gpeval.hip's translation unit
LIB_HEADERS = ("lower_core.h", "host_pool.h", "bigint_host.h", "trig_dev.h", "exact_int.h",
               "rccl_layer.h", "select_dev.h", "ctx.h", "fb_kernels.h", "asm_kernels.h",
               "planner.h", "exact_run.h")


def needs_build():
    if not os.path.exists(OUT):
        return True
    deps = [SRC, os.path.join(REPO, "include", "gpeval.h"), __file__, GEN,
            GEN32] + [os.path.join(HERE, "csrc", h) for h in LIB_HEADERS] + ASM_OUT + ASM32_OUT
    return any(os.path.getmtime(d) > os.path.getmtime(OUT) for d in deps)


NAT_SRC = os.path.join(HERE, "csrc", "flatten_native.cpp")
NAT_OUT = os.path.join(HERE, "_flatnative" +
                       sysconfig.get_config_var("EXT_SUFFIX"))


def build_native(force=False, verbose=False):
    """The native host flattener (CPython extension, g++)."""
    deps = [NAT_SRC, os.path.join(HERE, "csrc", "lower_core.h"),
            os.path.join(HERE, "csrc", "host_pool.h")]
    if not force and os.path.exists(NAT_OUT) and \
            all(os.path.getmtime(NAT_OUT) >= os.path.getmtime(d) for d in deps):
        return NAT_OUT
    cmd = ["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-Wall", "-pthread",
           "-I" + sysconfig.get_paths()["include"], NAT_SRC,
           "-o", NAT_OUT + ".tmp"]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(NAT_OUT + ".tmp", NAT_OUT)
    return NAT_OUT


def build(force=False, verbose=False):
    build_native(force, verbose)
    generate()
    if not force and not needs_build():
        return OUT
    cmd = [HIPCC] + FLAGS + [SRC, "-o", OUT + ".tmp"]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
