"""Run bench.py with native A/B setters applied first (measured-once knobs not on the bench CLI).

    python scripts/ab_native.py nhwc_wgrad_set_target=256 -- --model resnet50 --dtype bf16 --batch 32
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    argv = sys.argv[1:]
    cut = argv.index("--") if "--" in argv else len(argv)
    sets, rest = argv[:cut], argv[cut + 1:]
    from mxddp import native

    C = native()
    for kv in sets:
        k, v = kv.split("=", 1)
        getattr(C, k)(int(v))
        print(f"[ab_native] {k}({v})", file=sys.stderr)
    import bench

    sys.argv = ["bench.py"] + rest
    bench.main()


if __name__ == "__main__":
    main()
