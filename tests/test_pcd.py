"""PCD I/O: the global map files of mapOptmization.h:245-260 / :495-519.

Parity unpinned: the reference ships no .pcd files and PCL is not in this image, so the reader and
writer are checked against the published PCD v0.7 format (header keys, DATA ascii / binary /
binary_compressed with LZF and field-major layout) and against savePCDFileASCII's output rules
(PCL header text, 8 significant digits, "nan").  Host-only: these run without a GPU, except the
last test, which loads a map through fbr_load_map on the device.
"""
import os
import struct

import numpy as np
import pytest

from feature_base_pointcloud_registration_amd import api
from feature_base_pointcloud_registration_amd.fbr_types import POINT_XYZI, default_params

PCL_HEADER = ("# .PCD v0.7 - Point Cloud Data file format\nVERSION 0.7\nFIELDS x y z intensity\n"
              "SIZE 4 4 4 4\nTYPE F F F F\nCOUNT 1 1 1 1\nWIDTH {n}\nHEIGHT 1\n"
              "VIEWPOINT 0 0 0 1 0 0 0\nPOINTS {n}\nDATA {d}\n")


def _cloud(n, seed=0):
    rng = np.random.default_rng(seed)
    c = np.zeros(n, POINT_XYZI)
    for k, s in zip("xyz", (80.0, 80.0, 8.0)):
        c[k] = (rng.standard_normal(n) * s).astype(np.float32)
    c["intensity"] = rng.integers(0, 256, n).astype(np.float32)
    return c


def _bits(a):
    return np.ascontiguousarray(a).view(np.uint8)


def lzf_compress(data: bytes) -> bytes:
    """Greedy LZF encoder (liblzf's stream format), test-side only: literal runs <= 32 bytes,
    back references of 3..264 bytes within 8 KiB."""
    out, lit, i, n = bytearray(), bytearray(), 0, len(data)
    last = {}

    def flush():
        for s in range(0, len(lit), 32):
            chunk = lit[s:s + 32]
            out.append(len(chunk) - 1)
            out.extend(chunk)
        lit.clear()

    while i < n:
        best_len, best_off = 0, 0
        if i + 3 <= n:
            cand = last.get(data[i:i + 3])
            if cand is not None and i - cand <= 8192:
                ln = 0
                while i + ln < n and ln < 264 and data[cand + ln] == data[i + ln]:
                    ln += 1
                if ln >= 3:
                    best_len, best_off = ln, i - cand - 1
        if i + 3 <= n:
            last[data[i:i + 3]] = i
        if best_len:
            flush()
            ln = best_len - 2
            if ln < 7:
                out.append((ln << 5) | (best_off >> 8))
            else:
                out.append((7 << 5) | (best_off >> 8))
                out.append(ln - 7)
            out.append(best_off & 0xFF)
            for k in range(1, best_len):
                if i + k + 3 <= n:
                    last[data[i + k:i + k + 3]] = i + k
            i += best_len
        else:
            lit.append(data[i])
            i += 1
    flush()
    return bytes(out)


def lzf_decompress(data: bytes, size: int) -> bytes:
    out, i = bytearray(), 0
    while i < len(data):
        c = data[i]
        i += 1
        if c < 32:
            out.extend(data[i:i + c + 1])
            i += c + 1
        else:
            ln = c >> 5
            if ln == 7:
                ln += data[i]
                i += 1
            back = ((c & 0x1F) << 8) + data[i] + 1
            i += 1
            for _ in range(ln + 2):
                out.append(out[-back])
    assert len(out) == size
    return bytes(out)


def test_lzf_encoder_round_trip():
    rng = np.random.default_rng(3)
    for data in (b"", b"a", b"abcabcabcabcabcabc" * 40, bytes(rng.integers(0, 4, 5000, dtype=np.uint8)),
                 bytes(1000)):
        assert lzf_decompress(lzf_compress(data), len(data)) == data


def test_binary_round_trip_exact(tmp_path):
    c = _cloud(1537)
    c["x"][5] = np.nan
    c["y"][7] = -0.0
    p = tmp_path / "m.pcd"
    api.pcd_write(p, c, binary=True)
    raw = p.read_bytes()
    hdr = PCL_HEADER.format(n=len(c), d="binary").encode()
    assert raw[:len(hdr)] == hdr and len(raw) == len(hdr) + 16 * len(c)
    back = api.pcd_read(p)
    assert back.dtype == POINT_XYZI and np.array_equal(_bits(back), _bits(c))


def test_ascii_matches_save_pcd_file_ascii(tmp_path):
    c = _cloud(400, seed=1)
    c["z"][3] = np.nan
    c["x"][4] = 1e-7
    c["y"][9] = 123456789.0
    p = tmp_path / "cloudCorner.pcd"
    api.pcd_write(p, c)
    text = p.read_text()
    assert text.startswith(PCL_HEADER.format(n=len(c), d="ascii"))
    lines = text.splitlines()[11:]
    assert len(lines) == len(c)

    def fmt(v):
        return "nan" if np.isnan(v) else "%.8g" % float(v)

    for i in (0, 3, 4, 9, 399):
        assert lines[i] == " ".join(fmt(c[k][i]) for k in ("x", "y", "z", "intensity"))
    back = api.pcd_read(p)
    for k in ("x", "y", "z", "intensity"):
        exp = np.array([np.float32(float(fmt(v))) for v in c[k]], np.float32)
        assert np.array_equal(back[k], exp, equal_nan=True), k


def _write_raw(path, fields, sizes, types, counts, n, data_kind, body, extra_header=""):
    hdr = ("# generated\nVERSION .7\nFIELDS {}\nSIZE {}\nTYPE {}\nCOUNT {}\nWIDTH {}\nHEIGHT 1\n"
           "VIEWPOINT 0 0 0 1 0 0 0\n{}POINTS {}\nDATA {}\n").format(
        " ".join(fields), " ".join(map(str, sizes)), " ".join(types), " ".join(map(str, counts)), n,
        extra_header, n, data_kind)
    path.write_bytes(hdr.encode() + body)


# a non-PointXYZI layout: padding, doubles, an rgb word, a 3-count normal, intensity as u16
LAYOUT = dict(fields=["_", "x", "y", "z", "rgb", "normal", "intensity"],
              sizes=[4, 8, 4, 4, 4, 4, 2], types=["U", "F", "F", "F", "U", "F", "U"],
              counts=[1, 1, 1, 1, 1, 3, 1])
REC = np.dtype([("pad", "<u4"), ("x", "<f8"), ("y", "<f4"), ("z", "<f4"), ("rgb", "<u4"),
                ("normal", "<f4", 3), ("intensity", "<u2")])


def _layout_records(n, seed):
    rng = np.random.default_rng(seed)
    r = np.zeros(n, REC)
    r["pad"] = 0xDEADBEEF
    r["x"] = rng.standard_normal(n) * 50
    r["y"] = (rng.standard_normal(n) * 50).astype(np.float32)
    r["z"] = (rng.standard_normal(n) * 5).astype(np.float32)
    r["rgb"] = rng.integers(0, 2 ** 24, n)
    r["normal"] = rng.standard_normal((n, 3)).astype(np.float32)
    r["intensity"] = rng.integers(0, 65536, n)
    return r


def _check_layout(back, r):
    assert np.array_equal(back["x"], r["x"].astype(np.float32))
    assert np.array_equal(back["y"], r["y"]) and np.array_equal(back["z"], r["z"])
    assert np.array_equal(back["intensity"], r["intensity"].astype(np.float32))


def test_binary_other_field_layout(tmp_path):
    r = _layout_records(301, 4)
    p = tmp_path / "l.pcd"
    _write_raw(p, n=len(r), data_kind="binary", body=r.tobytes(), **LAYOUT)
    _check_layout(api.pcd_read(p), r)


def test_ascii_other_field_layout(tmp_path):
    r = _layout_records(57, 5)
    rows = []
    for q in r:
        rows.append(" ".join([str(q["pad"]), repr(float(q["x"])), "%.9g" % q["y"], "%.9g" % q["z"],
                              str(q["rgb"]), *("%.9g" % v for v in q["normal"]), str(q["intensity"])]))
    p = tmp_path / "l.pcd"
    _write_raw(p, n=len(r), data_kind="ascii", body=("\n".join(rows) + "\n").encode(), **LAYOUT)
    _check_layout(api.pcd_read(p), r)


def test_binary_compressed_field_major(tmp_path):
    r = _layout_records(777, 6)
    r["z"][::3] = 0.0  # give LZF something to match
    # binary_compressed stores the fields one after another (all x, then all y, ...)
    parts = [np.ascontiguousarray(r[name]).tobytes() for name in REC.names]
    raw = b"".join(parts)
    comp = lzf_compress(raw)
    body = struct.pack("<II", len(comp), len(raw)) + comp
    p = tmp_path / "c.pcd"
    _write_raw(p, n=len(r), data_kind="binary_compressed", body=body, **LAYOUT)
    _check_layout(api.pcd_read(p), r)


def test_missing_intensity_reads_zero(tmp_path):
    xyz = np.arange(30, dtype=np.float32).reshape(10, 3)
    p = tmp_path / "xyz.pcd"
    _write_raw(p, ["x", "y", "z"], [4, 4, 4], ["F", "F", "F"], [1, 1, 1], 10, "binary", xyz.tobytes())
    back = api.pcd_read(p)
    assert np.array_equal(back["x"], xyz[:, 0]) and np.array_equal(back["z"], xyz[:, 2])
    assert not back["intensity"].any()


def test_empty_cloud(tmp_path):
    p = tmp_path / "e.pcd"
    api.pcd_write(p, np.zeros(0, POINT_XYZI))
    assert p.read_text() == PCL_HEADER.format(n=0, d="ascii")
    assert len(api.pcd_read(p)) == 0
    api.pcd_write(p, np.zeros(0, POINT_XYZI), binary=True)
    assert len(api.pcd_read(p)) == 0


@pytest.mark.parametrize("case", ["missing_file", "no_xyz", "truncated_binary", "short_ascii",
                                  "bad_lzf_size", "points_mismatch", "unknown_data"])
def test_errors(tmp_path, case):
    p = tmp_path / "bad.pcd"
    F4 = dict(sizes=[4, 4, 4, 4], types=["F"] * 4, counts=[1] * 4)
    if case == "missing_file":
        p = tmp_path / "nope.pcd"
    elif case == "no_xyz":
        _write_raw(p, ["a", "b", "c", "d"], n=1, data_kind="binary", body=bytes(16), **F4)
    elif case == "truncated_binary":
        _write_raw(p, list("xyz") + ["intensity"], n=4, data_kind="binary", body=bytes(60), **F4)
    elif case == "short_ascii":
        _write_raw(p, list("xyz") + ["intensity"], n=2, data_kind="ascii", body=b"1 2 3 4\n5 6 7\n", **F4)
    elif case == "bad_lzf_size":
        raw = bytes(32)
        comp = lzf_compress(raw)
        _write_raw(p, list("xyz") + ["intensity"], n=2, data_kind="binary_compressed",
                   body=struct.pack("<II", len(comp), 31) + comp, **F4)
    elif case == "points_mismatch":
        _write_raw(p, list("xyz") + ["intensity"], n=2, data_kind="binary", body=bytes(64), **F4,
                   extra_header="")
        p.write_bytes(p.read_bytes().replace(b"POINTS 2", b"POINTS 3"))
    elif case == "unknown_data":
        _write_raw(p, list("xyz") + ["intensity"], n=1, data_kind="binary_lz4", body=bytes(16), **F4)
    with pytest.raises(api.FbrError) as e:
        api.pcd_read(p)
    assert e.value.status == -1


def test_capacity_error(tmp_path):
    import ctypes
    from feature_base_pointcloud_registration_amd.fbr_types import ptr
    p = tmp_path / "m.pcd"
    api.pcd_write(p, _cloud(10), binary=True)
    out = np.zeros(9, POINT_XYZI)
    n = ctypes.c_int64()
    assert api.lib().fbr_pcd_read(os.fsencode(p), ptr(out), 9, ctypes.byref(n)) == -4
    assert n.value == 10


@pytest.mark.gpu
def test_load_map_equals_set_map(tmp_path):
    from feature_base_pointcloud_registration_amd import synth
    corner, surf = synth.prior_map(seed=11)
    pc, ps = tmp_path / "cloudCorner.pcd", tmp_path / "cloudSurf.pcd"
    api.pcd_write(pc, corner, binary=True)
    api.pcd_write(ps, surf, binary=True)
    P = default_params(16, 1800)
    with api.Context(P) as a, api.Context(P) as b:
        a.set_map(corner, surf)
        b.load_map(pc, ps)
        for x, y in zip(a.get_map(), b.get_map()):
            assert np.array_equal(_bits(x), _bits(y))
        with pytest.raises(api.FbrError):
            b.load_map(tmp_path / "none.pcd", ps)
