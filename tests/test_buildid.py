"""Source fingerprint that ties committed PMC profiles to rebuilt binaries (buildid.py)."""
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from buildid import source_fingerprint  # noqa: E402


def _copy_sources(dst):
    pkg = os.path.join(dst, "cudatracerlib_amd")
    shutil.copytree(os.path.join(ROOT, "cudatracerlib_amd", "csrc"), os.path.join(pkg, "csrc"))
    shutil.copy(os.path.join(ROOT, "cudatracerlib_amd", "Makefile"), pkg)
    os.makedirs(os.path.join(dst, "include"))
    shutil.copy(os.path.join(ROOT, "include", "ctl_trace.h"), os.path.join(dst, "include"))


def test_fingerprint_is_location_independent_and_content_sensitive(tmp_path):
    _copy_sources(str(tmp_path))
    assert source_fingerprint(str(tmp_path)) == source_fingerprint(ROOT)
    with open(os.path.join(str(tmp_path), "cudatracerlib_amd", "csrc", "device", "traverse.h"), "a") as f:
        f.write("\n")
    assert source_fingerprint(str(tmp_path)) != source_fingerprint(ROOT)
