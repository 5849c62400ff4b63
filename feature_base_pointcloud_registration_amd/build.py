"""Build the in-tree native libraries.

  libfbr_hip.so    the product: HIP kernels for gfx950 + the extern "C" boundary (include/fbr.h)
  libfbr_synth.so  host-only synthetic scan/map generator (inputs for tests and bench.py)

Everything is compiled with -ffp-contract=off: the reference is plain x86-64 code without FMA, and
the kernels restate its float arithmetic operation by operation.
"""
import concurrent.futures
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
REPO = os.path.dirname(HERE)
OBJ = os.path.join(HERE, "build")

HIP_SOURCES = ["k_project.hip", "k_features.hip", "k_voxel.hip", "k_register.hip", "k_knn_r1.hip", "k_knn_r1f.hip",
               "k_knn_r2.hip", "k_knn_r2f.hip", "k_knn_r4.hip", "k_knn_r4f.hip", "k_knn_tile.hip", "k_keyframe.hip", "k_grid.hip",
               "k_selftest.hip", "fbr_api.hip"]
HOST_SOURCES = ["fbr_pcd.cpp", "fbr_msg.cpp", "fbr_imu.cpp"]  # host-only C++ in the same library (PCD, PointCloud2, IMU)
ARCH = os.environ.get("FBR_OFFLOAD_ARCH", "gfx950")


def hipcc():
    for cand in ("/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found")


def _newer(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _headers():
    hs = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    hs.append(os.path.join(REPO, "include", "fbr.h"))
    return hs


def build_hip(verbose=False, force=False, defines=(), name="libfbr_hip.so"):
    # one object directory per define set: a diagnostic variant never reuses another's objects
    obj_dir = OBJ if not defines else OBJ + "_" + "_".join(sorted(d.lower() for d in defines))
    os.makedirs(obj_dir, exist_ok=True)
    out = os.path.join(HERE, name)
    hdrs = _headers()
    flags = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", f"--offload-arch={ARCH}",
             "-I", CSRC, "-I", os.path.join(REPO, "include"), "-Wno-unused-result",
             *[f"-D{d}" for d in defines]]
    objs, jobs = [], []
    for src in HIP_SOURCES:
        s = os.path.join(CSRC, src)
        o = os.path.join(obj_dir, src.replace(".hip", ".o"))
        objs.append(o)
        if force or _newer(o, [s] + hdrs):
            jobs.append([hipcc(), *flags, "-c", s, "-o", o])
    for src in HOST_SOURCES:
        s = os.path.join(CSRC, src)
        o = os.path.join(obj_dir, os.path.splitext(src)[0] + ".o")
        objs.append(o)
        if force or _newer(o, [s] + hdrs):
            jobs.append(["g++", "-O2", "-std=c++17", "-fPIC", "-Wall", "-I", CSRC, "-I", os.path.join(REPO, "include"),
                         *[f"-D{d}" for d in defines], "-c", s, "-o", o])

    def run(cmd):
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        return r.stderr

    with concurrent.futures.ThreadPoolExecutor(max_workers=min(8, max(1, len(jobs)))) as ex:
        for err in ex.map(run, jobs):
            if verbose and err.strip():
                print(err)
    if force or jobs or _newer(out, objs):
        run([hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", out, *objs])
    return out


def build_synth(force=False):
    src = os.path.join(CSRC, "fbr_synth.cpp")
    out = os.path.join(HERE, "libfbr_synth.so")
    if force or _newer(out, [src, os.path.join(REPO, "include", "fbr.h")]):
        subprocess.check_call(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-o", out, src])
    return out


def build_all(verbose=False, force=False):
    return build_hip(verbose, force), build_synth(force)


if __name__ == "__main__":
    print(build_all(verbose="-v" in sys.argv, force="-f" in sys.argv))
