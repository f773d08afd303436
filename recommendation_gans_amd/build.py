"""Build librg_hip.so in-tree with hipcc for gfx950 (no JIT cache, no pip install).

    python -m recommendation_gans_amd.build        # or __graft_entry__.build()

The library is a plain C-ABI shared object (include/rg_hip.h) loaded with
ctypes; it is linked against the HIP runtime by SONAME (libamdhip64.so.7), so
inside a process that imported torch first it binds to the runtime torch
already loaded.
"""
import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIB = os.path.join(PKG, "librg_hip.so")
ARCH = os.environ.get("RG_OFFLOAD_ARCH", "gfx950")

SOURCES = ["rg_api.cpp", "rg_sampler.hip", "rg_mf.hip", "rg_stepper.cpp", "rg_comm.cpp", "rg_mtjump.cpp", "rg_ncf.hip",
           "rg_gemm.hip", "rg_gan.hip", "rg_eval.hip", "rg_plan.hip", "rg_owner.hip", "rg_uniform.hip", "rg_membw.hip",
           "rg_pool.cpp"]
HEADERS = ["rg_common.h", "rg_gemm.h", "rg_mt.h", "rg_owner.h", "rg_mlp_update.h"]


def _hipcc():
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm toolchain required to build librg_hip.so)")


def _inputs():
    files = [os.path.join(CSRC, s) for s in SOURCES + HEADERS]
    files.append(os.path.join(ROOT, "include", "rg_hip.h"))
    files.append(os.path.abspath(__file__))
    return files


def up_to_date():
    if not os.path.exists(LIB):
        return False
    t = os.path.getmtime(LIB)
    return all(os.path.getmtime(f) <= t for f in _inputs())


DIAG_LIB = os.path.join(PKG, "librg_hip_diag.so")


def build(force=False, verbose=False, jobs=8, diag=False, variant=None, defines=(), only=None):
    """diag=True: librg_hip_diag.so with the RG_DIAG_STAMPS phase stamps (scripts only;
    the product never loads it).  variant=NAME: _variants/librg_hip_NAME.so built with the
    extra -D defines, for same-box A/B runs (scripts load it through RG_LIB).  only=[src, ...]
    (variants): compile just those sources with the defines and link the product's objects
    for the rest."""
    if variant:
        os.makedirs(os.path.join(PKG, "_variants"), exist_ok=True)
        lib = os.path.join(PKG, "_variants", f"librg_hip_{variant}.so")
    else:
        lib = DIAG_LIB if diag else LIB
    if not force and not diag and not variant and up_to_date():
        return LIB
    hipcc = _hipcc()
    objdir = os.path.join(PKG, f"_obj_{variant}" if variant else "_obj_diag" if diag else "_obj")
    os.makedirs(objdir, exist_ok=True)
    common = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-I", os.path.join(ROOT, "include"),
              "-Wall", "-Wno-unused-function", "-ffp-contract=fast"] + (["-DRG_DIAG_STAMPS"] if diag else []) + \
        (os.environ.get("RG_EXTRA_CFLAGS", "").split() if diag else []) + [f"-D{d}" for d in defines]
    procs, objs = [], []
    for s in SOURCES:
        src = os.path.join(CSRC, s)
        if variant and only and s not in only:
            objs.append(os.path.join(PKG, "_obj", s + ".o"))
            continue
        obj = os.path.join(objdir, s + ".o")
        objs.append(obj)
        lang = ["-x", "hip"] if s.endswith(".hip") else []
        cmd = [hipcc] + common + lang + ["-c", src, "-o", obj]
        if verbose:
            print(" ".join(cmd))
        procs.append((s, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)))
    failed = []
    for s, p in procs:
        out = p.communicate()[0].decode()
        if p.returncode != 0:
            failed.append((s, out))
        elif verbose and out.strip():
            print(out)
    if failed:
        raise RuntimeError("hipcc failed:\n" + "\n".join(f"--- {s}\n{o}" for s, o in failed))
    tmp = lib + ".tmp"
    # librccl.so.1 by SONAME: inside a process that imported torch it binds to the
    # RCCL torch already loaded (same library torch.distributed's "nccl" backend uses)
    cmd = [hipcc, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", tmp] + objs + \
        ["-L/opt/rocm/lib", "-lrccl"]
    subprocess.check_call(cmd)
    os.replace(tmp, lib)
    return lib


if __name__ == "__main__":
    var = sys.argv[sys.argv.index("--variant") + 1] if "--variant" in sys.argv else None
    defs = [a[2:] for a in sys.argv if a.startswith("-D")]
    only = sys.argv[sys.argv.index("--only") + 1].split(",") if "--only" in sys.argv else None
    print(build(force="--force" in sys.argv, verbose="-v" in sys.argv, diag="--diag" in sys.argv, variant=var,
                defines=defs, only=only))
