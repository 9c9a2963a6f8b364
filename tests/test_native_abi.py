"""The C-ABI library loads and exports every symbol include/dol_hip.h declares
(no compute calls: this runs without a GPU), and the product refuses CPU
tensors instead of falling back."""
import ctypes
import os
import re

import pytest
import torch

from dolhip import _native, ops


def _header_symbols():
    src = open(_native.HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[\w]+\s*\*?\s*(dol_\w+)\s*\(", src, flags=re.M)))


def test_header_declares_the_hot_path():
    syms = _header_symbols()
    for s in ("dol_mix_csr_f32", "dol_mix_ring_f32", "dol_prox_admm_sgd_f32", "dol_admm_dual_f32",
              "dol_ordered_mean_f32", "dol_ordered_sum_f32", "dol_last_error", "dol_version"):
        assert s in syms


def test_library_exports_every_declared_symbol():
    assert os.path.exists(_native.LIB_PATH), "build libdol_hip.so first (__graft_entry__.build())"
    L = ctypes.CDLL(_native.LIB_PATH)
    missing = [s for s in _header_symbols() if not hasattr(L, s)]
    assert not missing, missing
    # and the Python binding covers exactly the declared surface
    assert set(_native.SIGNATURES) == set(_header_symbols())


def test_version_and_error_string():
    L = _native.lib()
    assert L.dol_version() == 100
    assert isinstance(L.dol_last_error(), bytes)


def test_argument_errors_are_reported_without_launch():
    L = _native.lib()
    rc = L.dol_mix_ring_f32(None, 4, None, 4, 5, 4, None, None, None, None, None)
    assert rc == -1
    assert b"null pointer" in L.dol_last_error()
    rc = L.dol_ordered_mean_f32(None, 4, None, 0, 4, None, None)
    assert rc == -1 and b"m must be >= 1" in L.dol_last_error()
    assert L.dol_admm_dual_workspace_bytes(4, 1 << 20) > 0
    fake = 1 << 20  # never dereferenced: every call below fails its argument check first
    rc = L.dol_er_stochastic_f32(fake, 100, 100, 1.5, 7, None)
    assert rc == -1 and b"p outside" in L.dol_last_error()
    rc = L.dol_er_stochastic_f32(fake, 70000, 70000, 0.1, 7, None)
    assert rc == -1 and b"65535" in L.dol_last_error()
    rc = L.dol_er_stochastic_f32(fake, 10, 100, 0.1, 7, None)
    assert rc == -1 and b"ldw" in L.dol_last_error()
    rc = L.dol_mix_dense_split3_f32(fake, 8, fake + 4096, 8, fake, 8, 8, 8, 8, fake, 1 << 30, 0, None)
    assert rc == -1 and b"alias" in L.dol_last_error()
    rc = L.dol_mix_dense_split3_f32(fake, 8, fake + 4096, 8, fake + 8192, 8, 8, 8, 8, fake, 16, 0, None)
    assert rc == -1 and b"workspace" in L.dol_last_error()
    # only blocks dol_bank_alloc handed out are unmapped (checked before any HIP call)
    assert L.dol_bank_free(fake, 1 << 21) == -1 and b"not a dol_bank_alloc block" in L.dol_last_error()
    assert L.dol_bank_free(None, 1 << 21) == 0


def test_pm_stage_order_setter():
    L = _native.lib()
    assert L.dol_pm_set_stage_order(-1) == -1 and b"outside" in L.dol_last_error()
    prev = L.dol_pm_set_stage_order(32)
    assert L.dol_pm_set_stage_order(prev) == 32
    assert L.dol_ring_steps_set_variant(6) == -1 and b"outside" in L.dol_last_error()
    assert L.dol_ring_steps_set_variant(5) == 0 and L.dol_ring_steps_set_variant(0) == 5  # the LDS-DMA sweep
    prev = L.dol_ring_steps_set_variant(2)
    assert L.dol_ring_steps_set_variant(prev) == 2


def test_slab_entry_points_check_arguments():
    L = _native.lib()
    fake = 1 << 20  # never dereferenced
    assert L.dol_csr_slab_nk(1024) == 16 and L.dol_csr_slab_nk(65) == 2 and L.dol_csr_slab_nk(0) == 0
    assert L.dol_csr_slab_hdr_len(1000, 1024) == 8 * 16 * 129 + 2 * 8 * 128  # blocks, perm, inv
    assert L.dol_csr_slab_ent_len(100, 10, 130) == 2 * (100 + 3 * 10 * 3 + 160)  # <= 3 pads per (row, chunk)
    rc = L.dol_mix_csr_slab_f32(fake, 16, 8, fake, 16, 8, 16, None, fake, None)
    assert rc == -1 and b"null pointer" in L.dol_last_error()
    rc = L.dol_mix_csr_slab_f32(fake, 16, 8, fake, 16, 8, 16, fake, fake, None)
    assert rc == -1 and b"alias" in L.dol_last_error()
    rc = L.dol_mix_csr_slab_f32(fake, 18, 8, fake + 4096, 16, 8, 16, fake, fake, None)
    assert rc == -1 and b"multiples of 4" in L.dol_last_error()
    rc = L.dol_mix_csr_slab_f32(fake, 16, 8, fake + 4096, 16, 8, 15, fake + 8, fake, None)
    assert rc == -1 and b"aligned" in L.dol_last_error()
    rc = L.dol_mix_csr_slab_f32(fake + 4, 16, 8, fake + 4096, 16, 8, 16, fake, fake, None)
    assert rc == -1 and b"16-B aligned" in L.dol_last_error()
    rc = L.dol_dense_to_csr_f32(fake, 8, 8, 8, fake, fake, fake, 63, None)
    assert rc == -1 and b"capacity" in L.dol_last_error()
    rc = L.dol_dense_to_csr_f32(fake, 4, 8, 8, fake, fake, fake, 64, None)
    assert rc == -1 and b"ldw" in L.dol_last_error()
    rc = L.dol_dense_to_csr_f32(fake, 70000, 70000, 70000, fake, fake, fake, 1 << 40, None)
    assert rc == -1 and b"2^31" in L.dol_last_error()
    rc = L.dol_csr_slab_pack(None, fake, fake, 8, 8, 0, fake, fake, None)
    assert rc == -1 and b"null pointer" in L.dol_last_error()


def test_split3_workspace_sizes():
    L = _native.lib()
    full = L.dol_mix_dense_split3_workspace_bytes(1024, 1024, 101770, 0)
    lean = L.dol_mix_dense_split3_workspace_bytes(1024, 1024, 101770, 2 | 4)  # X_ROWS_PADDED | FUSE_X
    # W pieces: Kg x Mp x 48 B; X pieces: Kg x Pp x 48 B (Kg = K/8, rows / columns padded to 256)
    assert lean == 128 * 1024 * 48
    assert full == lean + 128 * 101888 * 48
    assert L.dol_mix_dense_split3_workspace_bytes(0, 5, 5, 0) == 0


def test_cpu_tensors_are_refused():
    x = torch.zeros(4, 8)
    with pytest.raises(_native.DolNativeError):
        ops.mix_ring(x, torch.zeros(4, 8), torch.ones(4), torch.ones(4))
    with pytest.raises(_native.DolNativeError):
        ops.prox_admm_sgd(x, torch.zeros(4, 8), lr=0.1)


def _asan_runtime():
    import glob
    hits = sorted(glob.glob("/opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so"))
    return hits[-1] if hits else None


def test_argument_validation_under_asan_ubsan():
    """SURVEY §5 sanitizer row: the host side of the C-ABI built with
    -fsanitize=address,undefined (csrc/Makefile `asan`; device code unchanged)
    rejects NULL / negative / overflowing / misaligned arguments of every entry
    point without a sanitizer report (tests/asan_abi_driver.py, in a subprocess
    with the ASan runtime preloaded)."""
    import subprocess
    import sys
    rt = _asan_runtime()
    if rt is None:
        pytest.skip("no clang ASan runtime in this image")
    lib = os.path.join(os.path.dirname(_native.LIB_PATH), "libdol_hip_asan.so")
    if not os.path.exists(lib):
        subprocess.run(["make", "-s", "-C", _native.CSRC, "asan"], check=True, capture_output=True)
    env = dict(os.environ, LD_PRELOAD=rt, ASAN_OPTIONS="detect_leaks=0:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1", HIP_VISIBLE_DEVICES="")
    here = os.path.dirname(os.path.abspath(__file__))
    r = subprocess.run([sys.executable, os.path.join(here, "asan_abi_driver.py"), lib, _native.PKG_ROOT],
                       env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    assert "asan-abi ok" in r.stdout
