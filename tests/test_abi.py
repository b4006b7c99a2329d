"""C-ABI boundary checks that need no GPU: the library loads and exports every entry
point declared in include/ebsdvae.h; the ctypes table matches the header."""
import os
import re
import subprocess

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "ebsdvae.h")
LIB = os.path.join(ROOT, "ebsd-vae_amd", "lib", "libebsdvae.so")


def header_symbols():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(ebsdvae_[a-z0-9_]+)\s*\(", txt)))


def _ensure_built():
    if not os.path.exists(LIB):
        import sys
        sys.path.insert(0, os.path.join(ROOT, "ebsd-vae_amd"))
        import build
        build.build(verbose=False)


def test_header_and_ctypes_table_agree():
    from latice import _native
    assert header_symbols() == sorted(_native.exported_symbols())


def test_library_exports_every_header_symbol():
    _ensure_built()
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r"\b(ebsdvae_[a-z0-9_]+)\b", out))
    missing = [s for s in header_symbols() if s not in exported]
    assert not missing, missing


def header_abi_version() -> int:
    """EBSDVAE_ABI_VERSION of include/ebsdvae.h (the binding's ABI_VERSION must equal it)."""
    m = re.search(r"#define\s+EBSDVAE_ABI_VERSION\s+(\d+)", open(HEADER).read())
    assert m, "include/ebsdvae.h defines EBSDVAE_ABI_VERSION"
    return int(m.group(1))


def test_library_loads_and_binds():
    _ensure_built()
    from latice import _native
    lib = _native.load()
    assert lib.ebsdvae_version() == _native.ABI_VERSION == header_abi_version()
    for name in _native.exported_symbols():
        assert hasattr(lib, name)
    # host-side shape queries run without a GPU
    assert _native.call("ebsdvae_conv3x3_stat_tiles", 128, 128, 32) == 128
    assert _native.call("ebsdvae_conv3x3_wgrad_slices", 256, 128, 128, 32, 32) > 0
    assert _native.call("ebsdvae_in_bwd_tiles", 128, 128, 32) == 16


def test_planners_reject_byte_ranges_past_32_bits():
    """The split conv and weight-gradient kernels address one image through 32-bit buffer
    descriptors (reads past the range return 0): the planners refuse shapes whose per-image
    byte range reaches 2^31 instead of computing zeros silently."""
    _ensure_built()
    from latice import _native
    from latice.engine import PIECES_F16
    for np_ in (2, 3, PIECES_F16):
        assert _native.call("ebsdvae_conv3x3_split_supported", 128, 128, 32, 32, np_) == 1
        assert _native.call("ebsdvae_conv3x3_split_supported", 2048, 2048, 128, 128, np_) == 0
    assert _native.call("ebsdvae_conv3x3_wgrad_split_slices", 256, 128, 128, 32, 32, PIECES_F16) > 0
    assert _native.call("ebsdvae_conv3x3_wgrad_split_slices", 1, 2048, 2048, 128, 128, PIECES_F16) < 0


def test_invalid_shapes_report_errors_without_gpu():
    _ensure_built()
    from latice import _native
    # rejected by argument validation before any launch
    with pytest.raises(RuntimeError, match="cin=3"):
        _native.call("ebsdvae_conv3x3_fwd", 1, None, 0, 1, None, 1, None, None, 2, 16, 16, 3, 32, None)
    with pytest.raises(RuntimeError, match="null pointer"):
        _native.call("ebsdvae_heads_fwd", *([None] * 14), 2, 128, 4, 16, None)


def test_host_asan_driver():
    """the library's host code (argument validation, shape / scratch-size
    queries, error strings, batched descriptors at and past their limits) under
    AddressSanitizer: ebsd-vae_amd/build.py --asan links the library objects, built with
    -Xarch_host -fsanitize=address, into tests/asan/abi_asan.cpp.  No GPU needed.
    (__graft_entry__.build() builds it; here it is rebuilt only if stale.)"""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "ebsd-vae_amd"))
    import build
    try:
        exe = build.build_asan(verbose=False)
    except RuntimeError as e:      # pragma: no cover - toolchain missing
        pytest.skip(f"hipcc unavailable: {e}")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0 and "AddressSanitizer" not in r.stderr, (r.stdout + r.stderr)[-4000:]
    assert "abi_asan: ok" in r.stdout


def test_query_entry_points_are_registered_as_queries():
    """Size / support queries return their value instead of a status: every one the signature
    table lists must be in _native.QUERIES, or N.call would raise on its (nonzero) answer."""
    from latice import _native as N
    suffixes = ("_ok", "_tiles", "_slices", "_bytes", "_work", "_supported", "_version")
    queries = {n for n in N.SIGNATURES if n.endswith(suffixes)}
    assert queries <= N.QUERIES, sorted(queries - N.QUERIES)
    # and they answer on a CPU-only host (no device call behind them)
    assert N.call("ebsdvae_conv3x3_fwd_split_first_ok", 128, 128, 32, 32, N.PIECES_F16
                  if hasattr(N, "PIECES_F16") else 16) == 1
