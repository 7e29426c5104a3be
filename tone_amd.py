"""Import shim: exposes the package directory ``t-one_amd/`` as the importable name ``tone_amd``.

``t-one_amd`` is not a valid Python identifier, so this module turns itself into that package
(a module with ``__path__`` is a package) and runs the package ``__init__``.
"""
import os as _os

__package__ = __name__
__path__ = [_os.path.join(_os.path.dirname(_os.path.abspath(__file__)), "t-one_amd")]
_init = _os.path.join(__path__[0], "__init__.py")
with open(_init, encoding="utf-8") as _f:
    exec(compile(_f.read(), _init, "exec"))
