"""Run a Python script in this process with a native SIGSEGV/SIGABRT backtrace printer loaded
(tools/libsegv_trace.so) and faulthandler on: `python3 tools/segv_run.py bench.py --args`.
Debug aid for the exit-time crash seen under rocprofv3; the script runs via runpy (no exec)."""
import atexit
import ctypes
import faulthandler
import os
import runpy
import sys

faulthandler.enable(all_threads=True)
_maps_out = os.environ.get("SEGV_RUN_MAPS")


@atexit.register
def _dump_maps():
    """The process's mappings at interpreter exit (before the C exit handlers run), so the raw
    addresses of a crash in those handlers can be resolved to library + offset afterwards."""
    if _maps_out:
        with open("/proc/self/maps") as f, open(_maps_out, "w") as g:
            g.write(f.read())

ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libsegv_trace.so"))
script = sys.argv[1]
sys.argv = sys.argv[1:]
sys.path.insert(0, os.path.dirname(os.path.abspath(script)))
runpy.run_path(script, run_name="__main__")
