"""Build libgympo_amd.so (HIP for gfx950) in-tree: gym_po_amd/libgympo_amd.so.

    python gym-po-taxi_amd/build.py [--debug] [--stamps] [--asan]

--asan: a host-sanitised copy, gym_po_amd/libgympo_amd_asan.so (AddressSanitizer + UndefinedBehaviorSanitizer on
the host code only: -fsanitize follows -Xarch_host; device code is built as usual). tools/asan_cpu.sh runs the CPU
test suite against it with the clang ASan runtime preloaded.

hipcc cross-compiles without a GPU. Sources: csrc/*.hip (+ the C ABI header in include/).
Rebuilds only when a source is newer than the library.
"""
import glob
import hashlib
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
OUT = os.path.join(HERE, "gym_po_amd", "libgympo_amd.so")
ARCH = os.environ.get("GP_OFFLOAD_ARCH", "gfx950")


def sources():
    return sorted(glob.glob(os.path.join(HERE, "csrc", "*.hip")))


def deps():
    return sources() + glob.glob(os.path.join(HERE, "csrc", "*.h")) + [os.path.join(ROOT, "include", "gym_po_amd.h")]


def up_to_date(key=None):
    """The library is newer than every source and was built with the same compiler and flags (`key`, kept in
    libgympo_amd.so.key): a changed GP_OFFLOAD_ARCH / HIPCC / --debug rebuilds it."""
    if not os.path.exists(OUT):
        return False
    if key is not None:
        try:
            with open(OUT + ".key") as f:
                if f.read().strip() != key:
                    return False
        except OSError:
            return False
    t = os.path.getmtime(OUT)
    return all(os.path.getmtime(d) <= t for d in deps())


def build(force=False, debug=False, verbose=True, stamps=False, asan=False):
    """Compile each csrc/*.hip to an object in parallel (one hipcc per source), then link the .so."""
    out = OUT.replace(".so", "_stamps.so") if stamps else (OUT.replace(".so", "_asan.so") if asan else OUT)
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    flags = [f"--offload-arch={ARCH}", "-std=c++17", "-fPIC", "-O1" if debug else "-O3", "-Wno-unused-result",
             "-I", os.path.join(ROOT, "include")]
    if stamps:  # diagnostic build: s_memtime phase stamps in the fused kernel (never benchmarked)
        flags.insert(0, "-DGP_STAMPS")
    if debug or asan:
        flags.append("-g")
    san = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined",
           "-Xarch_host", "-fno-omit-frame-pointer", "-Xarch_host", "-fno-sanitize-recover=undefined"]
    if asan:
        flags += san
    # objects are keyed on the compiler and every flag (arch included): a changed GP_OFFLOAD_ARCH / HIPCC never
    # links objects built for another target
    key = hashlib.sha1(" ".join([hipcc] + flags).encode()).hexdigest()[:10]
    if not force and not stamps and not asan and up_to_date(key):
        return OUT
    kind = "stamps" if stamps else ("asan" if asan else ("debug" if debug else "release"))
    objdir = os.path.join(HERE, "build", kind + "-" + key)
    os.makedirs(objdir, exist_ok=True)

    headers = [d for d in deps() if not d.endswith(".hip")]

    def compile_one(src):
        obj = os.path.join(objdir, os.path.basename(src).replace(".hip", ".o"))
        if (not force and os.path.exists(obj)
                and all(os.path.getmtime(d) <= os.path.getmtime(obj) for d in [src, __file__] + headers)):
            return obj  # this object is newer than its source, every header and this script's flags
        cmd = [hipcc] + flags + ["-c", src, "-o", obj]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
        return obj

    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
        objs = list(ex.map(compile_one, sources()))
    cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC"] + (["-shared-libsan", "-fsanitize=address,undefined"]
                                                                   if asan else []) + ["-o", out + ".tmp"] + objs
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    if out == OUT:
        with open(OUT + ".key", "w") as f:
            f.write(key + "\n")
    return out


if __name__ == "__main__":
    build(force="--force" in sys.argv, debug="--debug" in sys.argv, stamps="--stamps" in sys.argv,
          asan="--asan" in sys.argv)
