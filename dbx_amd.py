"""Import shim: `import dbx_amd` loads the package directory
`distributed-backtesting-exploration_amd/` (its name is not a Python identifier)."""
import importlib.util
import os
import sys

_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)),
                    "distributed-backtesting-exploration_amd")
_spec = importlib.util.spec_from_file_location("dbx_amd", os.path.join(_DIR, "__init__.py"),
                                               submodule_search_locations=[_DIR])
_mod = importlib.util.module_from_spec(_spec)
sys.modules["dbx_amd"] = _mod
_spec.loader.exec_module(_mod)
