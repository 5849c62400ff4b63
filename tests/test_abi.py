"""The C-ABI library loads and exports every symbol include/fbr.h declares; host-side helpers.

No GPU is needed: only symbol resolution, defaults, error strings, the host pose conversions and the
no-device error path are exercised (compute calls are covered by tests/test_gpu_parity.py).
"""
import ctypes
import os
import re

import numpy as np
import pytest

import pyoracle as O
from conftest import REPO, has_gpu
from feature_base_pointcloud_registration_amd import api
from feature_base_pointcloud_registration_amd.fbr_types import FbrParams, default_params, ptr


def header_symbols():
    src = open(os.path.join(REPO, "include", "fbr.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(fbr_[a-z0-9_]+)\s*\(", src)))


def test_every_declared_symbol_is_exported():
    lib = ctypes.CDLL(api.lib_path())
    syms = header_symbols()
    assert len(syms) >= 25
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing
    assert sorted(api.EXPORTED_SYMBOLS) == syms


def test_params_default_match_params_yaml():
    p = FbrParams()
    api.lib().fbr_params_default(ctypes.byref(p))
    ref = default_params(16, 1800, max_batch=1)
    for name, _ in FbrParams._fields_:
        a, b = getattr(p, name), getattr(ref, name)
        if name in ("crop_half", "reserved_"):
            assert list(a) == list(b), name
        else:
            assert a == b, name
    assert (p.n_scan, p.horizon_scan, p.edge_threshold, p.surf_threshold) == (16, 1800, 1.0, np.float32(0.1))
    assert (p.mapping_corner_leaf_size, p.mapping_surf_leaf_size, p.max_iterations) == (np.float32(0.2), np.float32(0.4), 30)


def test_strerror_and_abi_version():
    assert api.lib().fbr_abi_version() == 4
    for code in range(-7, 1):
        assert api.strerror(code) and api.strerror(code) != "unknown status"
    assert api.strerror(-99) == "unknown status"


def test_pose_conversions_match_pcl_restatement():
    rng = np.random.default_rng(4)
    for _ in range(2000):
        pose = np.concatenate([rng.uniform(-1.4, 1.4, 3), rng.uniform(-100, 100, 3)]).astype(np.float32)
        m1, m2 = api.affine_from_pose(pose), O.affine_from_pose(pose)
        assert np.array_equal(m1.view(np.int32), m2.view(np.int32))
        p1, p2 = api.pose_from_affine(m1), O.pose_from_affine(m1)
        assert np.array_equal(p1.view(np.int32), p2.view(np.int32))
        assert np.allclose(p1, pose, atol=2e-5)


@pytest.mark.skipif(has_gpu(), reason="a HIP device is present")
def test_create_without_device_fails_loudly():
    p = default_params(16, 1800)
    with pytest.raises(api.FbrError) as e:
        api.Context(p)
    assert e.value.status == -6  # FBR_ERR_NO_DEVICE: no silent CPU fallback


def test_missing_extension_raises(monkeypatch, tmp_path):
    monkeypatch.setattr(api, "_LIB", None)
    monkeypatch.setattr(api, "lib_path", lambda: str(tmp_path / "libfbr_hip.so"))
    with pytest.raises(RuntimeError, match="not built"):
        api.lib()
