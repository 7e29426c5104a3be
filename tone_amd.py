"""Import shim: exposes the package directory ``t-one_amd/`` as the importable name ``tone_amd``.

``t-one_amd`` is not a valid Python identifier.  Importing this module loads that directory as a
regular package through importlib (a spec with ``submodule_search_locations``, so ``tone_amd.model``
etc. resolve inside it) and puts the package in ``sys.modules`` under this name, which is what the
``import`` statement then returns.
"""
import importlib.util as _ilu
import os as _os
import sys as _sys

_dir = _os.path.join(_os.path.dirname(_os.path.abspath(__file__)), "t-one_amd")
_spec = _ilu.spec_from_file_location(__name__, _os.path.join(_dir, "__init__.py"), submodule_search_locations=[_dir])
_pkg = _ilu.module_from_spec(_spec)
_sys.modules[__name__] = _pkg
_spec.loader.exec_module(_pkg)
