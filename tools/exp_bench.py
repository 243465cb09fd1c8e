"""bench.py on the test build libvo_exp.so with its experimental kernels selected
(vo_exp_set(fused_octave, msac_eager)): re-measures an experimental path at the product's
current design point.  usage: exp_bench.py <fused_octave 0|1> <msac_eager 0|1> [bench.py args]"""
import os
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parent.parent
os.environ["VO_LIBPATH"] = str(ROOT / "r7020e-visual-odometry_amd" / "lib" / "libvo_exp.so")
sys.path.insert(0, str(ROOT))
import vo_amd  # noqa: E402,F401
from r7020e_visual_odometry_amd import vo  # noqa: E402

fo, me = int(sys.argv[1]), int(sys.argv[2])
vo.load_experimental_library().vo_exp_set(fo, me)
sys.argv = ["bench.py"] + sys.argv[3:]
import bench  # noqa: E402
bench.main()
