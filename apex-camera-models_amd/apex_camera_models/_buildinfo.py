"""Build identity of libacm.so, importable without torch (profiles/collect_pmc.py
loads this file directly)."""
import glob
import hashlib
import os

_PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def source_sha256() -> str:
    """sha256 over the sources and build recipe of libacm.so (csrc/*.hip,
    csrc/*.hpp, include/acm.h, the Makefile): identifies the kernel code a
    build came from.  hipcc builds are not byte-reproducible (the offload
    bundle embeds temporary names), so a rebuild of unchanged sources gets a
    new file hash but the same source hash (bench.py's traffic check)."""
    root = os.path.dirname(_PKG_ROOT)
    files = sorted(glob.glob(os.path.join(_PKG_ROOT, "csrc", "*.hip")) +
                   glob.glob(os.path.join(_PKG_ROOT, "csrc", "*.hpp")) +
                   [os.path.join(root, "include", "acm.h"), os.path.join(_PKG_ROOT, "Makefile")])
    h = hashlib.sha256()
    for f in files:
        h.update(os.path.relpath(f, root).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()


def lib_identity(lib_path: str) -> dict:
    """The library file's name and its acm_version() string, which names the
    compile-time variant (ACM_IEEE_MATH, diagnostic defines): a PMC summary
    is attributed to a rebuilt library only if both match (bench.py)."""
    import ctypes
    L = ctypes.CDLL(lib_path)
    L.acm_version.restype = ctypes.c_char_p
    return {"name": os.path.basename(lib_path), "version": L.acm_version().decode()}
