"""Build the native library in-tree: crowdnav_dsrnn_amd/lib/libcrowdnav_hip.so (gfx950).

Provenance: the library embeds `CN_SRC_HASH=<sha256 of the compile flags + every source it depends on>`
(returned by cn_version()). `_lib.lib()` refuses a library whose embedded hash differs from the hash of
the sources on disk, so a stale prebuilt binary can never stand in for the committed code.
"""
import hashlib
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
LIB_DIR = os.path.join(HERE, "lib")
LIB_PATH = os.path.join(LIB_DIR, "libcrowdnav_hip.so")
SOURCES = [os.path.join(HERE, "csrc", "cn_engine.hip"), os.path.join(HERE, "csrc", "cn_gru.hip")]
DEPS = SOURCES + [os.path.join(HERE, "csrc", "cn_math.h"), os.path.join(REPO, "include", "crowdnav.h"),
                  os.path.join(REPO, "include", "crowdnav_state.h")]
ARCH = os.environ.get("CN_OFFLOAD_ARCH", "gfx950")


def hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if c and (os.path.isabs(c) and os.path.exists(c) or not os.path.isabs(c)):
            return c
    raise RuntimeError("hipcc not found")


FLAGS = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-Wno-unused-result"]
# Per-source extra flags. The step kernel's RNG phase inlines ocml's sin / cos / acos: machine LICM hoists
# their f64 polynomial constants (and kernel-argument copies) to the RNG loop's preheader, where they hold
# ~40 VGPRs across the whole loop; at the 3-workgroups-per-CU cap (168 VGPRs) that forced 34 VGPRs of
# scratch spills whose stores reached HBM every launch (~5 MB per C2 launch). Without machine LICM the C2
# variant fits in 165 VGPRs with no spill and the kd-tree variant drops 212 -> 178 VGPRs. The GRU
# kernels keep the default pipeline.
SRC_FLAGS = {"cn_engine.hip": ["-mllvm", "-disable-machine-licm"]}
HASH_MARK = b"CN_SRC_HASH="


def source_hash():
    """sha256 over the target arch, the compile flags and the bytes of every dependency, in order."""
    h = hashlib.sha256()
    h.update(("%s|%s|%s|" % (ARCH, " ".join(FLAGS), sorted(SRC_FLAGS.items()))).encode())
    for d in DEPS:
        h.update(os.path.relpath(d, REPO).encode() + b"\0")
        with open(d, "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    return h.hexdigest()


def built_hash(path=LIB_PATH):
    """The source hash embedded in a built library (None if absent or unreadable)."""
    try:
        with open(path, "rb") as f:
            blob = f.read()
    except OSError:
        return None
    i = blob.find(HASH_MARK)
    if i < 0:
        return None
    return blob[i + len(HASH_MARK):i + len(HASH_MARK) + 64].decode("ascii", "replace")


def needs_build():
    return built_hash() != source_hash()


def build(force=False, verbose=False):
    if not force and not needs_build():
        return LIB_PATH
    os.makedirs(LIB_DIR, exist_ok=True)
    tmp = LIB_PATH + ".tmp%d" % os.getpid()
    objs = []
    try:
        procs = []
        for src in SOURCES:   # one object per source (its own flags), compiled side by side, then one link
            obj = "%s.%s.o" % (tmp, os.path.basename(src))
            cmd = ([hipcc(), "--offload-arch=" + ARCH] + FLAGS + SRC_FLAGS.get(os.path.basename(src), []) +
                   ['-DCN_SRC_HASH="%s"' % source_hash(), "-c", "-o", obj, src])
            if verbose:
                print(" ".join(cmd), file=sys.stderr)
            procs.append((subprocess.Popen(cmd), cmd))
            objs.append(obj)
        failed = [cmd for p, cmd in procs if p.wait() != 0]
        if failed:
            raise subprocess.CalledProcessError(1, failed[0])
        cmd = [hipcc(), "--offload-arch=" + ARCH, "-shared", "-fPIC", "-o", tmp] + objs
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)
    finally:
        for o in objs:
            if os.path.exists(o):
                os.remove(o)
    os.replace(tmp, LIB_PATH)
    return LIB_PATH


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
