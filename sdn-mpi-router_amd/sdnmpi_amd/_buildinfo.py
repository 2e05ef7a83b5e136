"""Build identity of libsdnroute.so.

The library embeds a SHA-256 over the exact inputs it was compiled from --
the product sources, the two headers and the compile flags -- and exports it
as ``sdnr_build_id()`` (also as the byte marker ``SDNR_BUILD_ID:<hex>``, so a
build script can read it without loading the library).  ``build()``
recompiles whenever the tree's id differs from the library's, and the
loader (``_native.library``) refuses a library whose id is not the tree's:
the binary that runs on the GPU box is the one HEAD's ``csrc/`` describes.
"""
import hashlib
import os
import re

_HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(_HERE)
CSRC = os.path.join(PKG, "csrc")
INCLUDE = os.path.join(os.path.dirname(PKG), "include")

# the product library: the kernels the route calls select, and nothing else
# (losing variants live under tools/diag/)
SOURCES = ("capi.hip", "dfs.hip", "shortest.hip", "apsp.hip", "routes.hip", "ecmp.hip",
           "incremental.hip")
HEADERS = (("csrc", "common.h"), ("include", "sdnroute.h"))
FLAGS = ("--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function")
MARKER = b"SDNR_BUILD_ID:"


def inputs(csrc=CSRC, include=INCLUDE):
    """(label, path) of every hashed input, in hashing order."""
    out = [("csrc/" + s, os.path.join(csrc, s)) for s in SOURCES]
    for where, name in HEADERS:
        out.append((where + "/" + name, os.path.join(csrc if where == "csrc" else include, name)))
    return out


def tree_build_id(csrc=CSRC, include=INCLUDE):
    """SHA-256 (hex) of the sources, headers and flags; None when the sources
    are not there (an installed package without its csrc/)."""
    h = hashlib.sha256()
    h.update(" ".join(FLAGS).encode())
    for label, path in inputs(csrc, include):
        if not os.path.exists(path):
            return None
        h.update(b"\0" + label.encode() + b"\0")
        with open(path, "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def file_build_id(lib_path):
    """The id embedded in a built library file (marker scan, no load), or None."""
    try:
        with open(lib_path, "rb") as f:
            blob = f.read()
    except OSError:
        return None
    m = re.search(re.escape(MARKER) + rb"([0-9a-f]{64})", blob)
    return m.group(1).decode() if m else None
