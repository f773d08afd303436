"""The C-ABI library builds, loads without a GPU, and exports every symbol
include/rg_hip.h declares (no compute calls here)."""
import ctypes
import os
import re

import pytest

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


CTYPES_MIRRORS = {
    "rg_mf_tables_t": "MFTables", "rg_mf_batch_t": "MFBatch", "rg_mf_work_t": "MFWork",
    "rg_mf_loss_t": "MFLoss", "rg_opt_t": "Opt", "rg_mf_mark_t": "MFMark", "rg_mt_gen_t": "MTGen",
    "rg_mf_owner_batch_t": "MFOwnerBatch", "rg_mf_stepper_config_t": "MFStepperConfig",
    "rg_mf_step_in_t": "MFStepIn", "rg_ncf_model_t": "NCFModel", "rg_ncf_work_t": "NCFWork",
    "rg_gan_dims_t": "GANDims", "rg_gan_model_t": "GANModel", "rg_gan_batch_t": "GANBatch",
    "rg_gan_noise_t": "GANNoise", "rg_mf_lazy_t": "MFLazy", "rg_mf_pipe_t": "MFPipe"}


def header_structs():
    """{typedef name: [field names in declaration order]} for every struct of include/rg_hip.h."""
    txt = open(os.path.join(ROOT, "include", "rg_hip.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    out = {}
    for m in re.finditer(r"typedef\s+struct\s+\w*\s*\{(.*?)\}\s*(\w+)\s*;", txt, flags=re.S):
        fields = []
        for decl in m.group(1).split(";"):
            decl = " ".join(decl.split())
            if not decl:
                continue
            # "const float *a, *b" / "int64_t n" / "void *masks[8]": names after the type
            head, *rest = decl.split(",")
            names = [head.split()[-1]] + [r.strip() for r in rest]
            fields += [re.sub(r"[\*\s]|\[.*\]", "", nm) for nm in names]
        out[m.group(2)] = fields
    return out


def test_every_header_struct_has_a_ctypes_mirror():
    assert set(header_structs()) == set(CTYPES_MIRRORS), set(header_structs()) ^ set(CTYPES_MIRRORS)


def test_struct_layouts_match_header():
    """Every ctypes mirror has the C compiler's size and, field by field, the same names
    and offsets (the GAN / NCF / owner structs cross the boundary on every call too)."""
    import subprocess
    import tempfile
    from recommendation_gans_amd import _lib
    structs = header_structs()
    lines = []
    for name, fields in sorted(structs.items()):
        lines.append(f'printf("{name} %zu", sizeof({name}));')
        for f in fields:
            lines.append(f'printf(" %zu", offsetof({name}, {f}));')
        lines.append('printf("\\n");')
    src = "#include <stdio.h>\n#include <stddef.h>\n#include \"rg_hip.h\"\nint main(void){" + "\n".join(lines) + \
        "return 0;}\n"
    with tempfile.TemporaryDirectory() as td:
        c = os.path.join(td, "s.c")
        open(c, "w").write(src)
        exe = os.path.join(td, "s")
        subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), c, "-o", exe])
        got = {}
        for ln in subprocess.check_output([exe]).decode().splitlines():
            name, *nums = ln.split()
            got[name] = [int(x) for x in nums]
    for name, fields in structs.items():
        cls = getattr(_lib, CTYPES_MIRRORS[name])
        cfields = [f[0] for f in cls._fields_]
        assert cfields == fields, (name, cfields, fields)
        want = [ctypes.sizeof(cls)] + [getattr(cls, f).offset for f in fields]
        assert got[name] == want, (name, got[name], want)


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


def test_ncf_launch_geometry():
    """Host-side shape functions (no GPU): the E = 64 MLP runs one wave per tile of
    rg_ncf_rows_per_tile(64, 0) rows (48 = 8 whole columns of 1 + 5 rows in the product; 32 in a
    -DRG_NCF_WAVE_ROWS=32 build), 4 waves per workgroup, at most 256 workgroups; the other towers
    and NeuMF keep the tile kernel's 32-row tiles and workgroup-per-tile count (capped by LDS)."""
    from recommendation_gans_amd import _lib
    L = _lib.load()
    wave = not (_lib.ab_build() and os.environ.get("RG_NCF_TILE") == "1")
    R = int(L.rg_ncf_rows_per_tile(64, 0))
    assert R in ((32, 48) if wave else (32,))
    assert L.rg_ncf_rows_per_tile(32, 0) == 32 and L.rg_ncf_rows_per_tile(16, 50) == 32
    tc = R // 6
    assert L.rg_ncf_cols_per_tile(5, 64, 0) == tc and L.rg_ncf_tiles(8192, 5, 64, 0) == -(-8192 // tc)
    assert L.rg_ncf_cols_per_tile(5, 32, 0) == 5 and L.rg_ncf_tiles(8192, 5, 32, 0) == 1639
    assert L.rg_ncf_cols_per_tile(1, 64, 0) == R // 2
    assert L.rg_ncf_blocks(8192, 5, 64, 0) == 256
    t1000 = -(-1000 // tc)
    assert L.rg_ncf_blocks(1000, 5, 64, 0) == ((t1000 + 3) // 4 if wave else 200)
    assert L.rg_ncf_blocks(20, 5, 64, 0) == (1 if wave else 4)
    assert L.rg_ncf_blocks(1000, 5, 16, 50) == 200   # NeuMF: the tile kernel, one workgroup per tile
    assert L.rg_ncf_blocks(8192, 5, 48, 0) == -1     # unsupported width


def test_product_library_is_not_the_ab_build():
    """The shipped librg_hip.so carries none of the measured-slower alternatives (DESIGN §7, A/B
    build): rg_build_flags() is 0, the pipelined step refuses before touching the GPU, and the
    A/B variant (when built) says so about itself."""
    from recommendation_gans_amd import _lib
    if os.environ.get("RG_LIB"):
        pytest.skip("RG_LIB points at a variant")
    L = _lib.load()
    assert L.rg_build_flags() == 0 and not _lib.ab_build()
    rc = L.rg_mf_pipe_step(None, None, None, None, None, None, None, None, None, None, None)
    assert rc != 0 and b"A/B build" in L.rg_last_error()
    ab = os.path.join(os.path.dirname(_lib.LIB_PATH), "_variants", "librg_hip_ab.so")
    if os.path.exists(ab):
        A = ctypes.CDLL(ab, mode=ctypes.RTLD_LOCAL)
        A.rg_build_flags.restype = ctypes.c_int32
        assert A.rg_build_flags() & _lib.RG_BUILD_AB
