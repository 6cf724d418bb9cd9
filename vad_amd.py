"""Import alias for the package directory `causal-learning-based-video-anomaly-detection_paper_code_raw_amd/`
(its name is not a Python identifier).  `import vad_amd` / `from vad_amd.cad import ...` resolve into it."""
import os as _os

_PKG_DIR = _os.path.join(_os.path.dirname(_os.path.abspath(__file__)),
                         "causal-learning-based-video-anomaly-detection_paper_code_raw_amd")
__path__ = [_PKG_DIR]
__package__ = __name__
if __spec__ is not None:
    __spec__.submodule_search_locations = __path__
with open(_os.path.join(_PKG_DIR, "__init__.py")) as _f:
    exec(compile(_f.read(), _os.path.join(_PKG_DIR, "__init__.py"), "exec"))
