"""Every HIPFM_* environment knob named anywhere in the sources is registered (utils/knobs.py),
and the package reads them only through the registry (one documented configuration surface)."""
import glob
import os
import re

from hipfm.utils.knobs import KNOBS, describe, knob

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "deepfm-tensorflow-distributed-training-on-sagemaker_amd")
NAME = re.compile(r"HIPFM_[A-Z0-9_]*[A-Z0-9]")


def _sources():
    pats = ["*.py", "deepfm-tensorflow-distributed-training-on-sagemaker_amd/**/*.py", "csrc/**/*.hip",
            "csrc/**/*.h", "csrc/**/*.cpp", "scripts/*.sh", "tools/*.py", "tests/*.py"]
    for p in pats:
        yield from glob.glob(os.path.join(ROOT, p), recursive=True)


def test_every_knob_is_registered():
    missing = {}
    for f in _sources():
        for n in NAME.findall(open(f, errors="replace").read()):
            if n not in KNOBS:
                missing.setdefault(n, os.path.relpath(f, ROOT))
    assert not missing, f"unregistered HIPFM_* knobs: {missing}"


def test_package_reads_knobs_through_the_registry():
    direct = re.compile(r"os\.environ(\.get)?[\[(]\s*[\"']HIPFM_")
    bad = [os.path.relpath(f, ROOT) for f in glob.glob(os.path.join(PKG, "**", "*.py"), recursive=True)
           if not f.endswith("knobs.py") and direct.search(open(f).read())]
    assert not bad, bad


def test_defaults_and_describe(monkeypatch):
    assert knob("HIPFM_SPARSE") == "fused" and knob("HIPFM_SWEEP_MODE") == "auto"
    monkeypatch.setenv("HIPFM_SPARSE", "seg")
    assert knob("HIPFM_SPARSE") == "seg"
    text = describe()
    assert all(n in text for n in KNOBS)
    assert {k.kind for k in KNOBS.values()} <= {"variant", "tuning", "harness"}
