"""Run a script against a timing-variant build of liblbwn.so (same-box A/B runs only; the product
always loads the in-tree lb-wavenet_amd/lbwn/liblbwn.so).

    python tools/with_lib.py <variant liblbwn.so> <script.py> [args...]

The variant is loaded first, so every later lbwn._lib.load() in the process returns it."""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'lb-wavenet_amd'))
sys.path.insert(0, ROOT)

if __name__ == '__main__':
    lib, script = sys.argv[1], sys.argv[2]
    from lbwn import _lib
    _lib.load(os.path.abspath(lib))
    sys.argv = [script] + sys.argv[3:]
    runpy.run_path(script, run_name='__main__')
