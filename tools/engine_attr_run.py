"""A/B runner: set DistillEngine attributes, then run a script as __main__.

    python tools/engine_attr_run.py side_teacher=0 side_wgrad=0 -- bench.py --no-cpu-baseline ...

Every engine the script builds gets the attributes right after __init__ (the same
switches tools/physics_bench.py exposes as flags), so one script serves both arms of a
same-box A/B (tools/gpu_call.sh ab with AB_SCRIPT_VAR)."""
import os
import runpy
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "linkless-link-prediction_amd"))


def main():
    argv = sys.argv[1:]
    cut = argv.index("--")
    sets = {}
    for kv in argv[:cut]:
        k, v = kv.split("=", 1)
        sets[k] = bool(int(v)) if v in ("0", "1") else v
    script, rest = argv[cut + 1], argv[cut + 2:]
    import llp_engine
    init = llp_engine.DistillEngine.__init__

    def init_with(self, *a, **kw):
        init(self, *a, **kw)
        for k, v in sets.items():
            if not hasattr(self, k):
                raise AttributeError(f"DistillEngine has no attribute {k}")
            setattr(self, k, v)
    llp_engine.DistillEngine.__init__ = init_with
    sys.argv = [script] + rest
    runpy.run_path(script, run_name="__main__")


if __name__ == "__main__":
    main()
