"""C-ABI checks that need no GPU: libbf.so loads, exports every symbol include/bf.h declares, the ctypes
prototypes agree with the header, and argument validation fails before touching a device."""
import ctypes
import os
import re

import pytest

from dpdk_dc_sand_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "bf.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    out = {}
    for m in re.finditer(r"^\s*(?:const\s+)?[\w\s\*]+?\b(bf_\w+)\s*\(([^;]*?)\)\s*;", text, flags=re.M | re.S):
        args = [a.strip() for a in m.group(2).split(",") if a.strip() and a.strip() != "void"]
        out[m.group(1)] = len(args)
    return out


def test_header_parses():
    decl = declared_functions()
    assert {"bf_coeff_gen", "bf_reorder", "bf_beamform", "bf_beamform_fused", "bf_requant"} <= set(decl)


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(_lib.LIB_PATH)
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, f"libbf.so lacks {missing}"


def test_prototypes_match_header():
    decl = declared_functions()
    assert set(decl) == set(_lib.PROTOTYPES), set(decl) ^ set(_lib.PROTOTYPES)
    for name, nargs in decl.items():
        assert len(_lib.PROTOTYPES[name][1]) == nargs, name


def test_abi_version_and_error_channel():
    lib = _lib.load()
    assert lib.bf_abi_version() == 302  # 3.2: bf_beamform_study_single_channel; 3.1: bf_scatter_plan (WIDE16 rejected)
    assert isinstance(_lib.last_error(), str)


def test_argument_validation_without_gpu():
    fake = 1 << 20  # 16-byte aligned, never dereferenced: validation fails first
    with pytest.raises(_lib.BeamformerError, match="multiple of 16"):
        _lib.call("bf_reorder", fake, fake, 1, 4, 4, 17, None)
    with pytest.raises(_lib.BeamformerError, match="bad shape"):
        _lib.call("bf_beamform", fake, fake, fake, 0, 2, 1, 1, 4, 1, 0, None)
    with pytest.raises(_lib.BeamformerError, match="delay_channels"):
        _lib.call("bf_beamform_fused", fake, fake, 3, fake, 1, 4, 16, 4, 1, 1024, 0, 1e-9, 0.0, 0.0, 0, 1.0, None)
    with pytest.raises(_lib.BeamformerError, match="null pointer"):
        _lib.call("bf_coeff_gen", None, None, 1, 1, 1, 1, 1, 1, 0, 1e-9, None)
    with pytest.raises(_lib.BeamformerError, match="misaligned"):
        _lib.call("bf_beamform_fused", fake + 1, fake, 1, fake, 1, 4, 16, 4, 1, 1024, 0, 1e-9, 0.0, 0.0, 0, 1.0, None)
    with pytest.raises(_lib.BeamformerError, match="unknown flags"):
        _lib.call("bf_beamform_fused", fake, fake, 1, fake, 1, 4, 16, 4, 1, 1024, 0, 1e-9, 0.0, 0.0, 64, 1.0, None)
    with pytest.raises(_lib.BeamformerError, match="null pointer"):
        _lib.call("bf_coeff_gen_time_study", None, fake, 0, 4, 4, 4, 4, 1e-7, 8192, None)
    with pytest.raises(_lib.BeamformerError, match="bad shape"):
        _lib.call("bf_coeff_gen_time_study", fake, fake, 0, 0, 4, 4, 4, 1e-7, 8192, None)
    with pytest.raises(_lib.BeamformerError, match="sample_period"):
        _lib.call("bf_coeff_gen_time_study", fake, fake, 0, 4, 4, 4, 4, 0.0, 8192, None)
    with pytest.raises(_lib.BeamformerError, match="misaligned"):
        _lib.call("bf_coeff_gen_time_study", fake + 4, fake, 0, 4, 4, 4, 4, 1e-7, 8192, None)
    with pytest.raises(_lib.BeamformerError, match="null pointer"):
        _lib.call("bf_beamform_study_single_channel", fake, None, fake, 4, 32, 4, 4, 1e-7, 8192, None)
    with pytest.raises(_lib.BeamformerError, match="multiple of 16"):
        _lib.call("bf_beamform_study_single_channel", fake, fake, fake, 4, 40, 4, 4, 1e-7, 8192, None)
    with pytest.raises(_lib.BeamformerError, match="above 2048"):
        _lib.call("bf_beamform_study_single_channel", fake, fake, fake, 4, 32, 4096, 4, 1e-7, 8192, None)
    with pytest.raises(_lib.BeamformerError, match="misaligned"):
        _lib.call("bf_beamform_study_single_channel", fake + 4, fake, fake, 4, 32, 4, 4, 1e-7, 8192, None)


def test_algorithmic_bytes():
    lib = _lib.load()
    B, C, T, A, M = 8, 4096, 256, 64, 16
    got = lib.bf_fused_algorithmic_bytes(B, C, T, A, M, 1, 0)
    assert got == 2 * A * 2 * C * T * B + 8 * M * 2 * C * T * B + 16 * A * M
    assert lib.bf_fused_algorithmic_bytes(B, C, T, A, M, 1, 1) == 2 * A * 2 * C * T * B + 2 * M * 2 * C * T * B + \
        16 * A * M


def test_missing_library_fails_loudly(tmp_path):
    with pytest.raises(OSError, match="no CPU fallback"):
        _lib.load(str(tmp_path / "libbf.so"))


def test_pipeline_argument_validation_without_gpu():
    h = ctypes.c_void_p()
    with pytest.raises(_lib.BeamformerError, match="depth"):
        _lib.call("bf_pipeline_create", ctypes.byref(h), 1, 4, 16, 4, 1, 64, 0, 1e-9, 0, 1.0, 1, 0)
    with pytest.raises(_lib.BeamformerError, match="multiple of 16"):
        _lib.call("bf_pipeline_create", ctypes.byref(h), 1, 4, 17, 4, 1, 64, 0, 1e-9, 0, 1.0, 1, 2)
    with pytest.raises(_lib.BeamformerError, match="null pointer"):
        _lib.call("bf_pipeline_create", None, 1, 4, 16, 4, 1, 64, 0, 1e-9, 0, 1.0, 1, 2)
    with pytest.raises(_lib.BeamformerError, match="null pipeline"):
        _lib.call("bf_pipeline_wait", None, 0, 1)
    assert _lib.load().bf_pipeline_destroy(None) == 0
    # the fused call's flag checks, at creation (not at the first submit)
    with pytest.raises(_lib.BeamformerError, match="unknown kernel path"):
        _lib.call("bf_pipeline_create", ctypes.byref(h), 1, 4, 16, 4, 1, 64, 0, 1e-9, 0x700, 1.0, 1, 2)
    with pytest.raises(_lib.BeamformerError, match="unknown workgroup order"):
        _lib.call("bf_pipeline_create", ctypes.byref(h), 1, 4, 16, 4, 1, 64, 0, 1e-9, 0x3000, 1.0, 1, 2)
    with pytest.raises(_lib.BeamformerError, match="overflows"):
        _lib.call("bf_pipeline_create", ctypes.byref(h), 1, 4, 16, 364, 1, 64, 0, 1e-9, _lib.FUSED_OUT_INT8, 1.0, 1, 2)


def test_kernel_path_and_contract_flags_are_validated():
    fake = 1 << 20
    args = [fake, fake, 1, fake, 1, 4, 16, 4, 1, 1024, 0, 1e-9, 0.0, 0.0]
    for retired in (0x200, 0x500, 0x600, 0x700):  # removed measured-slower kernels (0x500: WIDE16, accepted by ABI 2.0, rejected since 3.0)
        with pytest.raises(_lib.BeamformerError, match="unknown kernel path"):
            _lib.call("bf_beamform_fused", *args, retired, 1.0, None)
    with pytest.raises(_lib.BeamformerError, match="unknown workgroup order"):
        _lib.call("bf_beamform_fused", *args, 0x3000, 1.0, None)
    # Q14 int8 contract: more uint8 antennas than the int32 beam sums hold (A * 255 * 23171 >= 2^31) is refused
    big = [fake, fake, 1, fake, 1, 4, 16, 364, 1, 1024, 0, 1e-9, 0.0, 0.0]
    with pytest.raises(_lib.BeamformerError, match="overflows"):
        _lib.call("bf_beamform_fused", *big, _lib.FUSED_OUT_INT8, 1.0, None)


def test_template_int8_overflow_bound():
    from dpdk_dc_sand_amd.beamforming import FusedBeamformerTemplate
    FusedBeamformerTemplate(None, 1, 4, 64, 16, 363, 1, out_int8=True)
    FusedBeamformerTemplate(None, 1, 4, 64, 16, 724, 1, out_int8=True, sample_signed=True)
    with pytest.raises(ValueError, match="overflow"):
        FusedBeamformerTemplate(None, 1, 4, 64, 16, 364, 1, out_int8=True)
    with pytest.raises(ValueError, match="overflow"):
        FusedBeamformerTemplate(None, 1, 4, 64, 16, 725, 1, out_int8=True, sample_signed=True)
    FusedBeamformerTemplate(None, 1, 4, 64, 16, 364, 1, out_int8=True, int8_contract="f32")
    t = FusedBeamformerTemplate(None, 1, 4, 64, 16, 4, 2, out_int8=True, kernel_path="wide", workgroup_order="xcd")
    assert t.flags == _lib.FUSED_OUT_INT8 | _lib.FUSED_PATH["wide"] | _lib.FUSED_ORDER["xcd"]
    with pytest.raises(ValueError, match="kernel_path"):
        FusedBeamformerTemplate(None, 1, 4, 64, 16, 4, 2, kernel_path="fast")


def test_product_library_never_reads_the_environment():
    """Kernel choice and contract switches are explicit flags: the product libbf.so imports no getenv (the
    measurement knobs live in the BF_DIAG build only)."""
    import shutil
    import subprocess
    nm = shutil.which("nm") or "/opt/rocm/lib/llvm/bin/llvm-nm"
    out = subprocess.run([nm, "-D", "--undefined-only", _lib.LIB_PATH], capture_output=True, text=True, check=True)
    names = {line.split()[-1].split("@")[0] for line in out.stdout.splitlines() if line.strip()}
    assert "getenv" not in names and "secure_getenv" not in names
