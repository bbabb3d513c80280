"""bench.py under a faulthandler watchdog: dumps every thread's Python stack and exits if the
run has not finished after CF_FH_SECONDS (default 100) -- for locating a hang on the GPU box."""
import faulthandler
import os
import runpy
import sys

faulthandler.dump_traceback_later(float(os.environ.get("CF_FH_SECONDS", "100")), exit=True)
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.argv = [os.path.join(root, "bench.py")] + sys.argv[1:]
sys.path.insert(0, root)
runpy.run_path(sys.argv[0], run_name="__main__")
