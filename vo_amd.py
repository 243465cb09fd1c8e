"""Import shim: the package directory is named `r7020e-visual-odometry_amd/`
(not a valid Python identifier).  `import vo_amd` loads it as the module
`r7020e_visual_odometry_amd`."""
import importlib.util
import sys
from pathlib import Path

_NAME = "r7020e_visual_odometry_amd"
_ROOT = Path(__file__).resolve().parent / "r7020e-visual-odometry_amd"

if _NAME in sys.modules:
    _mod = sys.modules[_NAME]
else:
    _spec = importlib.util.spec_from_file_location(_NAME, _ROOT / "__init__.py",
                                                   submodule_search_locations=[str(_ROOT)])
    _mod = importlib.util.module_from_spec(_spec)
    sys.modules[_NAME] = _mod
    _spec.loader.exec_module(_mod)
sys.modules[__name__] = _mod
