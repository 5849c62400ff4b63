"""Test configuration.

Markers:
  gpu  -- needs a HIP device (MI355X); run with `pytest -m gpu` on the GPU box.
CPU tests (`-m "not gpu"`) cover the oracle against the golden fixtures and the third-party
behaviour it pins (glibc atan2f, libstdc++ std::sort), host logic, and the C-ABI library's exports.
"""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))
NATIVE = os.path.join(REPO, "tests", "native")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X)")


def _ensure_built():
    from feature_base_pointcloud_registration_amd import build
    import pyoracle
    if not os.path.exists(pyoracle.lib_path()):
        pyoracle.build()
    build.build_synth()
    build.build_hip()


@pytest.fixture(scope="session", autouse=True)
def built_libs():
    _ensure_built()


def build_probe(name):
    """Compile tests/native/<name>.cpp (host code including product headers) with hipcc."""
    from feature_base_pointcloud_registration_amd import build
    src = os.path.join(NATIVE, name + ".cpp")
    out_dir = os.path.join(NATIVE, "build")
    os.makedirs(out_dir, exist_ok=True)
    out = os.path.join(out_dir, "lib" + name + ".so")
    deps = [src] + [os.path.join(build.CSRC, f) for f in os.listdir(build.CSRC) if f.endswith(".h")]
    if not os.path.exists(out) or any(os.path.getmtime(d) > os.path.getmtime(out) for d in deps):
        subprocess.check_call([build.hipcc(), "-O2", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off",
                               "-I", build.CSRC, "-I", os.path.join(REPO, "include"), "-o", out, src])
    import ctypes
    return ctypes.CDLL(out)


@pytest.fixture(scope="session")
def probe_lib():
    return build_probe("host_probe")


def build_shard_demo():
    """Compile tests/native/shard_demo.cpp (a native host sharding a C4 batch over processes, the
    pose records all-gathered over RCCL through the C-ABI) with the host compiler against
    libfbr_hip.so and the HIP runtime (device memory for the gathered records)."""
    from feature_base_pointcloud_registration_amd import api
    src = os.path.join(NATIVE, "shard_demo.cpp")
    out_dir = os.path.join(NATIVE, "build")
    os.makedirs(out_dir, exist_ok=True)
    out = os.path.join(out_dir, "shard_demo")
    lib = api.lib_path()
    deps = [src, lib, os.path.join(REPO, "include", "fbr.h")]
    if not os.path.exists(out) or any(os.path.getmtime(d) > os.path.getmtime(out) for d in deps):
        libdir = os.path.dirname(lib)
        subprocess.check_call(["g++", "-O2", "-std=c++17", "-Wall", "-D__HIP_PLATFORM_AMD__", "-I", "/opt/rocm/include",
                               "-I", os.path.join(REPO, "include"), "-o", out, src, "-L", libdir,
                               "-l:" + os.path.basename(lib), "-L/opt/rocm/lib", "-lamdhip64",
                               "-Wl,-rpath," + libdir, "-Wl,-rpath,/opt/rocm/lib", "-Wl,-rpath-link,/opt/rocm/lib"])
    return out


def has_gpu():
    try:
        from feature_base_pointcloud_registration_amd import api
        return api.device_count() > 0
    except Exception:
        return False


def build_mirror_demo():
    """Compile tests/native/mirror_demo.cpp (the C++ host mirror include/fbr.hpp driving the
    reference's cloudHandler chain) with the host compiler against libfbr_hip.so."""
    from feature_base_pointcloud_registration_amd import api
    src = os.path.join(NATIVE, "mirror_demo.cpp")
    out_dir = os.path.join(NATIVE, "build")
    os.makedirs(out_dir, exist_ok=True)
    out = os.path.join(out_dir, "mirror_demo")
    lib = api.lib_path()
    deps = [src, lib, os.path.join(REPO, "include", "fbr.hpp"), os.path.join(REPO, "include", "fbr.h")]
    if not os.path.exists(out) or any(os.path.getmtime(d) > os.path.getmtime(out) for d in deps):
        libdir = os.path.dirname(lib)
        subprocess.check_call(["g++", "-O2", "-std=c++17", "-Wall", "-I", os.path.join(REPO, "include"), "-o", out, src,
                               "-L", libdir, "-l:" + os.path.basename(lib), "-Wl,-rpath," + libdir,
                               "-Wl,-rpath-link,/opt/rocm/lib"])
    return out
