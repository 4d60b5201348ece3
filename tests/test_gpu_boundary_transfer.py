"""The boundary's host transfers (spx_load / spx_load_rows / spx_get_tableau)
in both layouts, through the C-ABI: a tableau loaded and read back unchanged,
byte for byte (-0.0, NaN payloads and infinities included), for row- and
column-major host arrays with and without row padding (ld > width), ragged
shapes and a tall narrow tableau whose row-major transfer takes more than one
staging chunk and more than 65535 row tiles (spx_capi.hip transfer_rows)."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _ptr(a):
    ct = ctypes.c_int64 if a.dtype == np.int64 else ctypes.c_double
    return a.ctypes.data_as(ctypes.POINTER(ct))


def _tableau(rows, cols, seed):
    rng = np.random.default_rng(seed)
    T = rng.standard_normal((rows, cols))
    flat = T.reshape(-1)
    k = min(flat.size, 7)
    flat[:k] = [-0.0, np.inf, -np.inf, 0.0, 1e-310, -1e308, 3.0][:k]
    if flat.size > 11:  # a NaN with a payload: bytes must survive
        flat[11] = np.frombuffer(np.uint64(0x7FF8000000C0FFEE).tobytes(), dtype=np.float64)[0]
    return T


def _get(e, layout, ld):
    from simplex_amd import _lib as L
    rows, cols = e.m_local + 1, e.N
    if layout == L.SPX_ROW_MAJOR:
        out = np.full((rows, ld), 7.25)
    else:
        out = np.full((cols, ld), 7.25)
    e._check(e._lib.spx_get_tableau(e._ctx, _ptr(out), ld, layout), "spx_get_tableau")
    return out


@pytest.mark.parametrize("shape", [(2, 1), (2, 3), (33, 65), (257, 7), (70, 40001), (1030, 2049)])
@pytest.mark.parametrize("order", ["C", "F"])
@pytest.mark.parametrize("pad", [0, 5])
def test_load_and_read_back_bytes(shape, order, pad):
    from simplex_amd import _lib as L
    from simplex_amd.engine import DeviceTableau
    rows, cols = shape
    T = _tableau(rows, cols, rows * 131 + cols)
    basis = np.arange(rows - 1, dtype=np.int64)
    with DeviceTableau(0) as e:
        if order == "C":
            host = np.full((rows, cols + pad), -5.5)
            host[:, :cols] = T
            layout, ld = L.SPX_ROW_MAJOR, cols + pad
        else:
            host = np.full((cols, rows + pad), -5.5)
            host[:, :rows] = T.T
            layout, ld = L.SPX_COL_MAJOR, rows + pad
        e._check(e._lib.spx_load(e._ctx, _ptr(host), rows, cols, ld, layout, _ptr(basis)),
                 "spx_load")
        e._refresh_dims()
        want = T.tobytes()
        assert e.tableau().tobytes() == want
        # both output layouts, with padding: the pad elements are not written
        rm = _get(e, L.SPX_ROW_MAJOR, cols + 3)
        assert np.ascontiguousarray(rm[:, :cols]).tobytes() == want
        assert np.all(rm[:, cols:] == 7.25)
        cm = _get(e, L.SPX_COL_MAJOR, rows + 2)
        assert np.ascontiguousarray(cm[:, :rows].T).tobytes() == want
        assert np.all(cm[:, rows:] == 7.25)


def test_tall_narrow_row_major_crosses_the_tile_limit():
    """2,100,001 x 2: a row-major transfer of more than 65535 tiles of 32 rows
    (the grid's y limit caps a chunk) and of several chunks."""
    from simplex_amd.engine import DeviceTableau
    rows, cols = 2_100_001, 2
    T = _tableau(rows, cols, 5)
    basis = np.arange(rows - 1, dtype=np.int64)
    with DeviceTableau(0) as e:
        e.load(T, basis)
        assert e.tableau().tobytes() == T.tobytes()
