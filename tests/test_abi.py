"""The C-ABI library loads on a CPU-only host and exports every symbol include/evacx.h declares."""
import ctypes
import os
import re

from golden_util import ROOT


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "evacx.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(evx_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_header_symbols():
    from evacx import _lib
    L = _lib.lib()
    syms = declared_symbols()
    assert len(syms) >= 7
    for s in syms:
        assert hasattr(L, s), s
    assert set(_lib.EXPORTS) <= set(syms)


def test_host_seeding_matches_reference_vectors():
    import numpy as np
    from golden_util import load
    from evacx import _lib
    v = load("rng_vectors")
    seeds = [0, 1, 1234, 99999, 2**31 + 5]
    s = np.array(seeds, np.uint32)
    py = np.zeros((len(seeds), 625), np.uint32)
    nps = np.zeros((len(seeds), 625), np.uint32)
    _lib.check(_lib.lib().evx_seed_host(s.ctypes.data, len(seeds), py.ctypes.data, nps.ctypes.data), "seed")
    for i, sd in enumerate(seeds):
        assert np.array_equal(py[i], v[f"py_seed_{sd}"])
        assert np.array_equal(nps[i], v[f"np_seed_{sd}"])


def test_layout_descriptor_and_errors_without_gpu():
    from evacx import _lib
    L = _lib.lib()
    lay = _lib.evx_layout(L=36, W=30, P=150, R=1)
    # tables missing -> error code, message, no crash, no device touched
    rc = L.evx_env_step(ctypes.byref(lay), None, None, None, None)
    assert rc < 0 and b"table" in L.evx_last_error()
    assert L.evx_step_lds_bytes(ctypes.byref(lay)) == -1


def test_repel_threshold_exact():
    import math
    from evacx.env import repel_threshold
    for r in [5.0, 4.5, 0.3, 7.1, 12.0, 1e-3]:
        n = repel_threshold(r)
        assert math.sqrt(n) >= r and (n == 0 or math.sqrt(n - 1) < r)


def test_missing_library_fails_loudly(tmp_path):
    """No CPU fallback: a product call without libevacx.so raises EvacxError."""
    import subprocess
    import sys
    code = ("import sys; sys.path.insert(0, %r)\n"
            "from evacx import _lib\n"
            "try:\n    _lib.lib()\nexcept _lib.EvacxError as e:\n    print('raised', e)\n    sys.exit(0)\n"
            "sys.exit(3)\n") % os.path.join(ROOT, "dqn-marl_amd")
    env = dict(os.environ, EVX_LIB=str(tmp_path / "absent" / "libevacx.so"))
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "not built" in r.stdout
