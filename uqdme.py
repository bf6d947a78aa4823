"""Import alias for the package directory `unbiased-quantization-distributed-mean-estimation_amd/`
(a hyphenated name is not importable).  `import uqdme` loads it as `uqdme_amd` and
re-exports its public API, e.g. `from uqdme import Type_unbiased_quantize`."""
import importlib.util as _ilu
import os as _os
import sys as _sys

_PKG_NAME = "uqdme_amd"
_PKG_DIR = _os.path.join(_os.path.dirname(_os.path.abspath(__file__)),
                         "unbiased-quantization-distributed-mean-estimation_amd")

if _PKG_NAME in _sys.modules:
    _pkg = _sys.modules[_PKG_NAME]
else:
    _spec = _ilu.spec_from_file_location(_PKG_NAME, _os.path.join(_PKG_DIR, "__init__.py"),
                                         submodule_search_locations=[_PKG_DIR])
    _pkg = _ilu.module_from_spec(_spec)
    _sys.modules[_PKG_NAME] = _pkg
    _spec.loader.exec_module(_pkg)

PACKAGE_DIR = _PKG_DIR
__all__ = list(_pkg.__all__) + ["PACKAGE_DIR"]
globals().update({k: getattr(_pkg, k) for k in _pkg.__all__})
