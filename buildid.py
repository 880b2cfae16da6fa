"""Source fingerprint of libctl_trace.so.

hipcc's offload bundles are not byte-reproducible (two builds of the same
sources in different directories hash differently), so a profile recorded on
one build cannot be matched to a rebuild by the library hash alone.  The
fingerprint hashes what the library is compiled from: the Makefile, every
file under csrc/ and the C-ABI header.  bench.py reports a committed PMC
profile as belonging to the running binary when either the library hash or
this fingerprint matches (and says which).
"""
import hashlib
import os

_HERE = os.path.dirname(os.path.abspath(__file__))


def source_fingerprint(root=_HERE):
    pkg = os.path.join(root, "cudatracerlib_amd")
    files = [os.path.join(pkg, "Makefile"), os.path.join(root, "include", "ctl_trace.h")]
    for d, _, names in os.walk(os.path.join(pkg, "csrc")):
        files += [os.path.join(d, n) for n in names if n.endswith((".h", ".hip", ".cpp"))]
    h = hashlib.sha256()
    for f in sorted(files):
        h.update(os.path.relpath(f, root).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
        h.update(b"\0")
    return h.hexdigest()
