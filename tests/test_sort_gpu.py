"""The step kernel's key sort (wave_sort_keys: rank sort up to 64 keys, register bitonic up to 512,
512-key register blocks with memory passes beyond -- the contested list of a big grid's heavy env
reaches thousands of movers) through evx_diag_sort_keys, against numpy's sort of the same
distinct keys (target << pb | person, as the step builds them)."""
import ctypes as C

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n", [1, 63, 64, 100, 512, 513, 1000, 1024, 2500, 4096, 7000, 8193, 9102])
def test_step_key_sort_matches_numpy(n):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from evacx import _lib
    L = _lib.lib()
    L.evx_diag_sort_keys.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p]
    rng = np.random.default_rng(n)
    pb = 14  # person bits of a 9102-person layout
    targets = rng.integers(0, 66564, n, dtype=np.uint64)
    persons = rng.permutation(1 << pb)[:n].astype(np.uint64)
    keys = np.unique(((targets << pb) | persons).astype(np.uint32))
    rng.shuffle(keys)
    dev = torch.from_numpy(keys.view(np.int32).copy()).cuda()
    pad = torch.zeros(1 << int(np.ceil(np.log2(max(len(keys), 1)))), dtype=torch.int32, device="cuda")
    assert L.evx_diag_sort_keys(dev.data_ptr(), pad.data_ptr(), len(keys), None) == 0
    torch.cuda.synchronize()
    assert np.array_equal(dev.cpu().numpy().view(np.uint32), np.sort(keys))
