"""Import shim: the package lives in the directory ``datou-gomoku-muzero_amd/`` (a name Python
cannot import directly because of the hyphens).  ``import datou_gomoku_muzero_amd`` runs this file,
which loads that directory as the package ``datou_gomoku_muzero_amd`` and replaces itself in
``sys.modules`` so that ``import datou_gomoku_muzero_amd.engine`` etc. work normally."""
import importlib.util
import os
import sys

_PKG_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "datou-gomoku-muzero_amd")
_spec = importlib.util.spec_from_file_location(
    __name__, os.path.join(_PKG_DIR, "__init__.py"), submodule_search_locations=[_PKG_DIR])
_pkg = importlib.util.module_from_spec(_spec)
sys.modules[__name__] = _pkg
_spec.loader.exec_module(_pkg)
