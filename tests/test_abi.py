"""CPU: the C-ABI library (libdmf_hip.so) builds for gfx950, loads without a
GPU, exports exactly what include/dmf_hip.h declares, and reports argument
errors through dmf_last_error() (no compute call needs a device here).
Also: the product path refuses CPU tensors and a missing library loudly --
there is no CPU fallback."""
import ctypes
import os
import re
import subprocess
import sys

import pytest
import torch

import dmf_native as N

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.dirname(N.__file__)


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(N.LIB_PATH):
        subprocess.run(["make", "-C", os.path.join(PKG, "csrc"), "-j8"], check=True)
    return N.load()


def _exported(path):
    out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True, check=True).stdout
    return sorted({ln.split()[-1] for ln in out.splitlines() if re.search(r" T dmf_", ln)})


def test_header_declares_entry_points():
    syms = N.declared_symbols()
    assert len(syms) > 60
    for s in ("dmf_conv2d_fwd", "dmf_conv2d_dgrad", "dmf_conv2d_wgrad", "dmf_bn_finalize", "dmf_affine_act",
              "dmf_focal_loss", "dmf_soft_dice", "dmf_recon_loss", "dmf_mimic_loss", "dmf_adamw_multi",
              "dmf_attn_fwd", "dmf_mask_attn_fwd", "dmf_last_error", "dmf_abi_version"):
        assert s in syms, s


def test_library_exports_every_declared_symbol(lib):
    exported = _exported(N.LIB_PATH)
    declared = N.declared_symbols()
    assert sorted(set(declared) - set(exported)) == []
    # nothing exported under the dmf_ prefix that the header does not declare
    assert sorted(set(exported) - set(declared)) == []
    sigs = N._signatures()
    assert set(sigs) == set(declared)


def test_code_object_targets_gfx950(lib):
    with open(N.LIB_PATH, "rb") as f:
        blob = f.read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob
    assert b"gfx942" not in blob and b"gfx90a" not in blob


def test_abi_version(lib):
    with open(os.path.join(ROOT, "include", "dmf_hip.h")) as f:
        want = int(re.search(r"#define DMF_ABI_VERSION (\d+)", f.read()).group(1))
    assert lib.dmf_abi_version() == want


def test_argument_errors_are_reported(lib):
    # bad geometry is rejected before any HIP call: status -1 + message
    rc = lib.dmf_bn_finalize(None, 0, 0, 1.0, 1.0, None, None, None, None, None, 0.1, 1e-5, 1, None, None, None,
                             None)
    assert rc == -1
    assert b"dmf_bn_finalize" in lib.dmf_last_error()
    with pytest.raises(RuntimeError, match="dmf_bn_finalize"):
        N.call("dmf_bn_finalize", None, 0, 0, 1.0, 1.0, None, None, None, None, None, 0.1, 1e-5, 1, None, None,
               None, None)
    # large-T training finalize without a workspace is refused
    assert lib.dmf_bn_finalize_ws_size(1024, 128) == 0
    assert lib.dmf_bn_finalize_ws_size(1025, 128) == 33 * 128 * 2
    rc = lib.dmf_bn_finalize(ctypes.c_void_p(16), 2000, 8, 1.0, 1.0, None, None, None, None, None, 0.1, 1e-5, 1,
                             ctypes.c_void_p(16), None, None, None)
    assert rc == -1 and b"workspace" in lib.dmf_last_error()


def test_conv_shape_checks(lib):
    # Cin not a multiple of 8 on the MFMA path / zero batch are argument errors
    rc = lib.dmf_conv2d_fwd(1, None, 0, 8, 8, 16, 16, None, 0, 0, None, 16, 3, 3, 1, 1, 1, None, None, 8, 8, 16,
                            None, 0, None, 0, None)
    assert rc == -1
    assert lib.dmf_last_error()


def test_product_ops_refuse_cpu_tensors():
    import dmf_ops as O

    x = torch.randn(1, 8, 4, 4).to(memory_format=torch.channels_last)
    conv = torch.nn.Conv2d(8, 8, 3, padding=1)
    with pytest.raises(RuntimeError, match="no CPU fallback|device tensors"):
        O.conv2d(x, conv, {}, "none")


def test_missing_library_fails_loudly(tmp_path):
    code = ("import torch, sys; sys.path.insert(0, %r); import dmf_native as N\n"
            "try:\n    N.load()\nexcept RuntimeError as e:\n    print('ERR', e)\n" % PKG)
    env = dict(os.environ, DMF_HIP_LIB=str(tmp_path / "nope.so"))
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert "ERR HIP extension not built" in out.stdout, out.stdout + out.stderr
