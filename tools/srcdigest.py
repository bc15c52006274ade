"""Digest of the sources that build the product library (csrc/ + include/): profiles/*.json
written by the counter passes carry it, and bench.py compares it with the tree it runs from,
so a bench line never silently describes counters of older code.
Usable as a module (src_digest()) or a script (prints it)."""
import glob
import hashlib
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def src_digest(root: str = ROOT) -> str:
    files = sorted(glob.glob(os.path.join(root, "assignment-for-aae6102_gnss-sdr_amd", "csrc", "*")) +
                   glob.glob(os.path.join(root, "include", "*.h")))
    h = hashlib.sha256()
    for p in files:
        if os.path.isfile(p):
            h.update(os.path.relpath(p, root).encode())
            with open(p, "rb") as fh:
                h.update(fh.read())
    return h.hexdigest()[:16]


def head_commit(root: str = ROOT) -> str | None:
    """The commit the tree was sent from (.head_sha, written before each gpurun call), if any."""
    try:
        with open(os.path.join(root, ".head_sha")) as fh:
            return fh.read().strip() or None
    except OSError:
        return None


def stamp(d: dict, root: str = ROOT) -> dict:
    d["src_digest"] = src_digest(root)
    d["git_commit"] = head_commit(root)
    return d


if __name__ == "__main__":
    print(src_digest())
