"""Import alias for the framework package.

The framework's sources live in ``deepfm-tensorflow-distributed-training-on-sagemaker_amd/``
(a directory name that is not a valid Python identifier).  This shim makes that directory
importable as ``hipfm``: it points the package search path at it and executes its
``__init__`` in this module's namespace, so ``hipfm.ops``, ``hipfm.models`` ... resolve to
the files there under a single, consistent module name.
"""
import os as _os

_PKG_DIR = _os.path.join(
    _os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))),
    "deepfm-tensorflow-distributed-training-on-sagemaker_amd",
)
__path__ = [_PKG_DIR]
__file__ = _os.path.join(_PKG_DIR, "__init__.py")
with open(__file__) as _f:
    exec(compile(_f.read(), __file__, "exec"))
