"""The C-ABI library builds, loads without a GPU, and exports every symbol
include/rg_hip.h declares (no compute calls here)."""
import ctypes
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    names = set()
    for fn in os.listdir(os.path.join(ROOT, "include")):
        if not fn.endswith(".h"):
            continue
        txt = open(os.path.join(ROOT, "include", fn)).read()
        txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
        for m in re.finditer(r"^\s*(?:const\s+)?[A-Za-z_][\w\s\*]*?\b(rg_\w+)\s*\(", txt, flags=re.M):
            names.add(m.group(1))
    return names


def test_header_declares_functions():
    names = header_functions()
    assert {"rg_mt_generate", "rg_mf_pairs", "rg_mf_apply", "rg_mf_scores", "rg_last_error"} <= names


def test_library_exports_all_header_symbols():
    from recommendation_gans_amd import build
    path = build.build()
    lib = ctypes.CDLL(path)
    missing = [n for n in sorted(header_functions()) if not hasattr(lib, n)]
    assert not missing, missing


def test_python_binding_covers_header():
    from recommendation_gans_amd import _lib
    bound = {n for n, _, _ in _lib.SIGNATURES}
    assert header_functions() <= bound, header_functions() - bound
    L = _lib.load()
    assert b"gfx950" in L.rg_version()


def test_struct_layouts_match_header():
    """ctypes mirrors of the structs have the sizes the C compiler gives them."""
    import subprocess
    import tempfile
    from recommendation_gans_amd import _lib
    src = r'''
#include <stdio.h>
#include "rg_hip.h"
int main(void){printf("%zu %zu %zu %zu %zu %zu %zu\n", sizeof(rg_mf_tables_t), sizeof(rg_mf_batch_t),
 sizeof(rg_mf_work_t), sizeof(rg_opt_t), sizeof(rg_mf_loss_t), sizeof(rg_mf_stepper_config_t),
 sizeof(rg_mf_step_in_t)); return 0;}
'''
    with tempfile.TemporaryDirectory() as td:
        c = os.path.join(td, "s.c")
        open(c, "w").write(src)
        exe = os.path.join(td, "s")
        subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), c, "-o", exe])
        sizes = [int(x) for x in subprocess.check_output([exe]).split()]
    assert sizes == [ctypes.sizeof(_lib.MFTables), ctypes.sizeof(_lib.MFBatch),
                     ctypes.sizeof(_lib.MFWork), ctypes.sizeof(_lib.Opt), ctypes.sizeof(_lib.MFLoss),
                     ctypes.sizeof(_lib.MFStepperConfig), ctypes.sizeof(_lib.MFStepIn)]


def test_no_gpu_means_loud_failure():
    import torch
    if torch.cuda.is_available():
        return
    from recommendation_gans_amd import _lib
    try:
        _lib.require_gpu()
    except RuntimeError as e:
        assert "GPU" in str(e)
    else:
        raise AssertionError("require_gpu must raise without a GPU")
