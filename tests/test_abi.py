"""The C-ABI library loads and exports every symbol include/tvq.h declares (CPU only)."""
import ctypes
import os
import re

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "tvq.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(tvq_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_functions():
    names = declared_functions()
    assert "tvq_vq_assign" in names and "tvq_last_error" in names


def test_library_exports_every_declared_symbol():
    from timevqvae.hip import _native
    if not os.path.exists(_native.LIB_PATH):
        pytest.fail(f"{_native.LIB_PATH} missing: run __graft_entry__.build()")
    h = ctypes.CDLL(_native.LIB_PATH)
    missing = [n for n in declared_functions() if not hasattr(h, n)]
    assert not missing, missing
    h.tvq_abi_version.restype = ctypes.c_int
    assert h.tvq_abi_version() >= 1


def test_binding_covers_every_declared_symbol():
    from timevqvae.hip import _native
    extra = {"tvq_last_error", "tvq_abi_version"}
    missing = [n for n in declared_functions() if n not in _native.SIGNATURES and n not in extra]
    assert not missing, missing


def test_product_refuses_cpu_tensors():
    import torch
    from timevqvae.hip._native import NativeError, ptr
    with pytest.raises(NativeError):
        ptr(torch.zeros(3))


def test_library_stamp_matches_sources():
    """The library carries the hash of the sources it was built from (csrc/Makefile
    tvq_source_hash); __graft_entry__.build() rebuilds when it differs, so the library the
    GPU tests load is the tree's."""
    from timevqvae.hip import _native
    assert _native.built_hash() == _native.source_hash(), (
        f"libtvq_hip.so was built from other sources ({_native.built_hash()} vs "
        f"{_native.source_hash()}): run __graft_entry__.build()")


@pytest.mark.gpu
def test_mapped_library_is_the_trees(cuda):
    """On the GPU box: the libtvq_hip.so this process actually mapped (after a kernel ran
    through it) is the in-tree file, and its compiled-in stamp -- asked of the mapped library
    itself, not read from the file -- equals the hash of the sources in this tree."""
    import torch
    from timevqvae.hip import _native
    h = _native.lib()
    x = torch.zeros(64, device=cuda)
    _native.call("tvq_fill", _native.ptr(x), 64, 1.5, _native.stream_ptr())
    torch.cuda.synchronize()
    assert float(x.sum()) == 96.0
    mapped = sorted({ln.split()[-1] for ln in open("/proc/self/maps")
                     if ln.rstrip().endswith("libtvq_hip.so")})
    assert mapped == [os.path.realpath(_native.LIB_PATH)], mapped
    stamp = h.tvq_source_hash().decode()
    assert stamp == _native.source_hash(), f"mapped library {stamp} != sources {_native.source_hash()}"
    print(f"mapped {mapped[0]} stamp {stamp} extra '{h.tvq_build_extra().decode()}'")
