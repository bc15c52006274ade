"""Digest of the sources that build the product library (csrc/ + include/): profiles/*.json
written by the counter passes carry it, and bench.py compares it with the tree it runs from,
so a bench line never silently describes counters of older code.
Usable as a module (src_digest()) or a script (prints it)."""
import glob
import hashlib
import os
import subprocess

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


def git_head(root: str = ROOT) -> str | None:
    """`git rev-parse HEAD` (+ "-dirty" when tracked files differ from it), where the tree has
    its .git (here; gpurun snapshots leave it behind)."""
    try:
        h = subprocess.run(["git", "-C", root, "rev-parse", "HEAD"], capture_output=True, text=True, timeout=10)
        if h.returncode != 0:
            return None
        d = subprocess.run(["git", "-C", root, "status", "--porcelain", "--untracked-files=no"],
                           capture_output=True, text=True, timeout=20)
        return h.stdout.strip() + ("-dirty" if d.returncode == 0 and d.stdout.strip() else "")
    except (OSError, subprocess.SubprocessError):
        return None


def head_commit(root: str = ROOT) -> str | None:
    """The commit of the running tree: git itself where .git exists, else .head_sha (written by
    __graft_entry__.build() and before each gpurun call from `git rev-parse HEAD`)."""
    g = git_head(root)
    if g:
        return g
    try:
        with open(os.path.join(root, ".head_sha")) as fh:
            return fh.read().strip() or None
    except OSError:
        return None


def head_commit_source(root: str = ROOT) -> str:
    return "git" if git_head(root) else ".head_sha"


def write_head_sha(root: str = ROOT) -> None:
    g = git_head(root)
    if g:
        with open(os.path.join(root, ".head_sha"), "w") as fh:
            fh.write(g + "\n")


def file_digest(path: str) -> str | None:
    """sha256 (16 hex) of a built file, e.g. the product library a process loaded."""
    try:
        h = hashlib.sha256()
        with open(path, "rb") as fh:
            for blk in iter(lambda: fh.read(1 << 20), b""):
                h.update(blk)
        return h.hexdigest()[:16]
    except OSError:
        return None


def stamp(d: dict, root: str = ROOT) -> dict:
    d["src_digest"] = src_digest(root)
    d["git_commit"] = head_commit(root)
    return d


if __name__ == "__main__":
    print(src_digest())
