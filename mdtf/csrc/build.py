"""Build the native libraries in-tree.

* ``mdtf/csrc/build/libmdtf_kernels.so`` — HIP/CDNA4 kernels (``*.hip``),
  ``hipcc --offload-arch=gfx950 -O3``; C ABI, loaded by ``mdtf/ops/_native.py``.
* ``mdtf/csrc/build/libmdtf_host.so`` — host C++ (CRC32C, TFRecord I/O,
  threaded shuffling loader), ``g++ -O3 -msse4.2``.

Each source is compiled to an object file only when it (or a header) changed;
objects compile in parallel.  Usage: ``python -m mdtf.csrc.build [--clean]``.
"""
import concurrent.futures
import glob
import hashlib
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "build")
ARCH = os.environ.get("MDTF_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

HIP_FLAGS = ["-O3", "-std=c++17", "--offload-arch=%s" % ARCH, "-fPIC", "-munsafe-fp-atomics",
             "-Wno-unused-result", "-I", os.path.join(HERE, "include")]
HOST_FLAGS = ["-O3", "-std=c++17", "-msse4.2", "-fPIC", "-pthread", "-Wall", "-Wno-unused-result"]


def _digest(paths, extra):
    h = hashlib.sha1()
    for p in sorted(paths):
        with open(p, "rb") as f:
            h.update(f.read())
    h.update(" ".join(extra).encode())
    return h.hexdigest()[:16]


def _headers():
    # shared headers and the kernel-template includes (conv_ws_kernel.inc is compiled by several .hip files)
    return glob.glob(os.path.join(HERE, "include", "*.h")) + glob.glob(os.path.join(HERE, "*.inc"))


def _compile_obj(src, flags, compiler):
    base = os.path.splitext(os.path.basename(src))[0]
    dig = _digest([src] + _headers(), flags + [compiler])
    obj = os.path.join(OUT, "%s.%s.o" % (base, dig))
    if os.path.exists(obj):
        return obj, False
    for stale in glob.glob(os.path.join(OUT, "%s.*.o" % base)):
        os.remove(stale)
    cmd = [compiler] + flags + ["-c", src, "-o", obj + ".tmp"]
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("compile failed: %s\n%s" % (" ".join(cmd), r.stdout))
    os.replace(obj + ".tmp", obj)
    return obj, True


def _link(objs, out, compiler, flags):
    cmd = [compiler] + flags + ["-shared", "-o", out + ".tmp"] + objs
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("link failed: %s\n%s" % (" ".join(cmd), r.stdout))
    os.replace(out + ".tmp", out)


def build(verbose=True, jobs=None):
    os.makedirs(OUT, exist_ok=True)
    jobs = jobs or min(8, os.cpu_count() or 4)
    results = {}
    # host library
    host_srcs = sorted(glob.glob(os.path.join(HERE, "host", "*.cpp")))
    hip_srcs = sorted(glob.glob(os.path.join(HERE, "*.hip")))
    with concurrent.futures.ThreadPoolExecutor(jobs) as ex:
        futs = {ex.submit(_compile_obj, s, HOST_FLAGS, "g++"): ("host", s) for s in host_srcs}
        futs.update({ex.submit(_compile_obj, s, HIP_FLAGS, HIPCC): ("hip", s) for s in hip_srcs})
        objs = {"host": [], "hip": []}
        for f in concurrent.futures.as_completed(futs):
            kind, src = futs[f]
            obj, fresh = f.result()
            objs[kind].append(obj)
            if verbose and fresh:
                print("[mdtf build] compiled %s" % os.path.relpath(src, HERE))
    host_lib = os.path.join(OUT, "libmdtf_host.so")
    if objs["host"]:
        _link(sorted(objs["host"]), host_lib, "g++", ["-pthread"])
        results["host"] = host_lib
    if objs["hip"]:
        hip_lib = os.path.join(OUT, "libmdtf_kernels.so")
        _link(sorted(objs["hip"]), hip_lib, HIPCC, ["--offload-arch=%s" % ARCH, "-fPIC"])
        results["kernels"] = hip_lib
    if verbose:
        print("[mdtf build] done: %s" % ", ".join("%s=%s" % (k, os.path.relpath(v, HERE)) for k, v in results.items()))
    return results


def clean():
    shutil.rmtree(OUT, ignore_errors=True)


if __name__ == "__main__":
    if "--clean" in sys.argv:
        clean()
    build()
