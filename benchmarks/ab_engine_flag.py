"""A/B one HipEngine class switch under bench.py: ``python -m benchmarks.ab_engine_flag FLAG VALUE
[bench.py args]`` sets ``HipEngine.FLAG = VALUE`` (int) before bench.py builds the engine."""
import sys

from distributed_tensorflow_for_dcgan_amd.engine.hip_engine import HipEngine


def main():
    flag, value = sys.argv[1], int(sys.argv[2])
    if not hasattr(HipEngine, flag):
        raise SystemExit("HipEngine has no switch %s" % flag)
    cur = getattr(HipEngine, flag)
    setattr(HipEngine, flag, bool(value) if cur is None or isinstance(cur, bool) else type(cur)(value))
    sys.argv = ["bench.py"] + sys.argv[3:]
    import bench
    bench.main()


if __name__ == "__main__":
    main()
