"""Hash of the native sources (csrc/, the Makefile, include/rtmi.h): sha256,
first 16 hex digits. The Makefile compiles it into librtmi.so
(rt_build_source_hash), PMC summaries record it, and bench.py / the tests
compare the loaded library's hash with the tree's. No imports beyond the
standard library: `python3 rtmi/srchash.py` prints it for the Makefile.
"""
import hashlib
import os


def source_hash(pkg=None):
    pkg = pkg or os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    files = [os.path.join(pkg, "Makefile"), os.path.join(os.path.dirname(pkg), "include", "rtmi.h")]
    csrc = os.path.join(pkg, "csrc")
    files += [os.path.join(csrc, f) for f in sorted(os.listdir(csrc)) if f.endswith((".h", ".hip", ".cpp"))]
    h = hashlib.sha256()
    for f in files:
        h.update(os.path.basename(f).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


if __name__ == "__main__":
    print(source_hash())
