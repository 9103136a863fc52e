"""In-tree build of libjwave_hip.so (gfx950) via jwave_amd/csrc/Makefile.

Provenance: every build writes ``lib/libjwave_hip.so.json`` next to the
library: the SHA-256 of the sources it was built from (csrc/ + include/), of
the library itself, the compiler and target.  A library is stale when that
source digest differs from the tree's (content, not mtimes: a copied tree
keeps its verdict), and ``_lib.lib()`` refuses to load a stale library when
it may not rebuild (JWAVE_AMD_NO_BUILD=1, as on the GPU box).
"""
import datetime
import hashlib
import json
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "lib", "libjwave_hip.so")
STAMP = LIB + ".json"


def _sources():
    out = []
    for d in (CSRC, os.path.join(HERE, "..", "include")):
        for f in os.listdir(d):
            if f.endswith((".hip", ".cpp", ".hpp", ".h")) or f == "Makefile":
                out.append(os.path.join(d, f))
    return sorted(out, key=os.path.basename)


def source_digest():
    h = hashlib.sha256()
    for p in _sources():
        h.update(os.path.basename(p).encode() + b"\0")
        with open(p, "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    return h.hexdigest()


def _file_digest(p):
    h = hashlib.sha256()
    with open(p, "rb") as f:
        for blk in iter(lambda: f.read(1 << 20), b""):
            h.update(blk)
    return h.hexdigest()


def stamp():
    """The provenance record of the in-tree library (None if absent)."""
    try:
        with open(STAMP) as f:
            return json.load(f)
    except (OSError, ValueError):
        return None


def stale():
    if not os.path.exists(LIB):
        return True
    s = stamp()
    return s is None or s.get("sources_sha256") != source_digest()


def _hipcc_version():
    try:
        out = subprocess.run(["/opt/rocm/bin/hipcc", "--version"], capture_output=True,
                             text=True, timeout=60).stdout
        return next((l.strip() for l in out.splitlines() if "clang version" in l), out[:80])
    except Exception:
        return None


def build(force=False, jobs=5):
    compiled = False
    was_stale = stale()
    if force or was_stale:
        before = os.path.getmtime(LIB) if os.path.exists(LIB) else None
        jobs = min(int(jobs), 16)
        subprocess.check_call(["make", "-s", "-j%d" % jobs, "-C", CSRC]
                              + (["-B"] if force else []))
        compiled = before is None or os.path.getmtime(LIB) != before
    s = stamp()
    # make is the judge of what to recompile (mtimes); the record follows
    # whenever the sources or the library differ from it
    if compiled or was_stale or s is None or s.get("lib_sha256") != _file_digest(LIB):
        rec = {"sources_sha256": source_digest(), "lib_sha256": _file_digest(LIB),
               "arch": "gfx950", "hipcc": _hipcc_version(),
               "built_utc": datetime.datetime.utcnow().strftime("%Y-%m-%dT%H:%M:%SZ"),
               "compiled_by_this_call": compiled}
        with open(STAMP, "w") as f:
            json.dump(rec, f, indent=1)
    return LIB
