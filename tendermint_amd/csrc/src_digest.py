"""Digest of the sources libtmgpu.so is built from (tmv_version's src=...).

The Makefile compiles it in; bench.py and smoke() recompute it over the
tree they run from and report whether the loaded library matches.
Usage: python3 src_digest.py [--git]   (prints the digest, or "<digest> <git HEAD>")
"""
import hashlib
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
INCLUDE = os.path.join(HERE, "..", "..", "include")
EXT = (".hip", ".h", ".cpp", ".py")


def source_files():
    out = []
    for root in (HERE, os.path.join(HERE, "host")):
        for f in sorted(os.listdir(root)):
            if f.endswith(EXT) or f == "Makefile":
                out.append(os.path.join(root, f))
    for f in sorted(os.listdir(INCLUDE)):
        if f.endswith(".h"):
            out.append(os.path.join(INCLUDE, f))
    return out


def digest(n: int = 16) -> str:
    h = hashlib.sha256()
    for p in source_files():
        h.update(os.path.relpath(p, HERE).encode() + b"\0")
        with open(p, "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    return h.hexdigest()[:n]


def git_head() -> str:
    try:
        r = subprocess.run(["git", "-C", HERE, "rev-parse", "--short=12", "HEAD"], capture_output=True, text=True,
                           timeout=10)
        head = r.stdout.strip() if r.returncode == 0 else "none"
        d = subprocess.run(["git", "-C", HERE, "status", "--porcelain", "--", ".", "../../include"],
                           capture_output=True, text=True, timeout=10)
        return head + ("+dirty" if d.returncode == 0 and d.stdout.strip() else "")
    except Exception:
        return "none"


if __name__ == "__main__":
    print(digest() + (" " + git_head() if "--git" in sys.argv else ""))
