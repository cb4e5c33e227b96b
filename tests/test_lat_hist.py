"""The verify tile's native tsorig -> tspub histogram
(fd_verify_tile_lat_publish, include/fd_verify_tile.h): 1-us bins below
32.768 ms, 64-us bins above up to 2.13 s, an overflow count past that; the
Python summary (firedancer_amd.tile.LatHist) reads percentiles at bin
centres.  Host-only: the callback is called directly, no GPU."""
import ctypes

import numpy as np

from firedancer_amd import lib
from firedancer_amd.tile import LAT_BINS, LatHist, lat_bin_ms


def publish(h, d_ns):
    f = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_ulong, ctypes.c_void_p, ctypes.c_ulong,
                         ctypes.c_ulong, ctypes.c_ulong, ctypes.c_ulong)(h.fn.value)
    for d in d_ns:
        f(h.ctx, 0, None, 0, 0, 1_000_000_000, 1_000_000_000 + int(d))


def test_bins_cover_two_seconds():
    lib()
    h = LatHist()
    publish(h, [500, 1_500, 32_767_999, 32_768_000, 32_768_000 + 64_000 * 5 + 10, 2_000_000_000, 3_000_000_000])
    b = h.buf[4:]
    assert b[0] == 1 and b[1] == 1 and b[32767] == 1 and b[32768] == 1 and b[32768 + 5] == 1
    assert b[(32768 + (2_000_000 - 32768) // 64)] == 1
    assert b[LAT_BINS - 1] == 1 and h.buf[3] == 1          # 3 s: the overflow bin
    s = h.summary()
    assert s["count"] == 7 and abs(s["max_ms"] - 3000.0) < 1e-9 and s["over_2s"] == 1


def test_percentiles_at_large_latencies():
    lib()
    h = LatHist()
    rng = np.random.default_rng(5)
    d = rng.uniform(60e6, 100e6, 2000)       # 60-100 ms: all past the 1-us range
    publish(h, d)
    s = h.summary()
    assert abs(s["p50_ms"] - np.percentile(d, 50) * 1e-6) < 0.2
    assert abs(s["p99_ms"] - np.percentile(d, 99) * 1e-6) < 0.2
    assert s["over_2s"] == 0
    assert abs(lat_bin_ms(100) - 0.1005) < 1e-12 and abs(lat_bin_ms(32768) - 32.8) < 1e-9
