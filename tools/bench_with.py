"""bench.py with module attributes of the package set first (same-process A/B of executor choices that have no
environment switch):  python tools/bench_with.py unet_exec._FUSE_ENC_OUT=False -- [bench.py args]"""
import importlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    argv = sys.argv[1:]
    cut = argv.index("--") if "--" in argv else len(argv)
    for a in argv[:cut]:
        target, val = a.split("=", 1)
        mod, attr = target.rsplit(".", 1)
        m = importlib.import_module("superresolution_for_pdes_amd." + mod)
        setattr(m, attr, eval(val, {}, {}))
    sys.argv = [os.path.join(ROOT, "bench.py")] + argv[cut + 1:]
    import bench
    bench.main()


if __name__ == "__main__":
    main()
