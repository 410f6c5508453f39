"""Source hash of libencx.so: sha256 over every file the library is built from.

`make` bakes it into the library (`encx_build_id()`, build/buildid.c) and `encx._lib` recomputes
it from the sources next to the library at load time, refusing a library built from other
sources (a stale `.so` pushed to a GPU box once ran tests against code it was not built from).
Standalone (no torch import): `python3 buildid.py` prints the hash for the Makefile.
"""
import glob
import hashlib
import os

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)


def sources():
    """Every input of libencx.so, as (name relative to the repo root, absolute path), sorted."""
    files = glob.glob(os.path.join(PKG, 'csrc', '*.hip')) + glob.glob(os.path.join(PKG, 'csrc', '*.h'))
    files.append(os.path.join(ROOT, 'include', 'encx.h'))
    return sorted((os.path.relpath(f, ROOT), f) for f in files)


def build_id():
    h = hashlib.sha256()
    for rel, path in sources():
        with open(path, 'rb') as f:
            data = f.read()
        h.update(rel.encode() + b'\0' + str(len(data)).encode() + b'\0' + data)
    return h.hexdigest()[:32]


if __name__ == '__main__':
    print(build_id())
