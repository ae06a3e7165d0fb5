"""Interleaved A/B timing of kernel variants on any bench leg -- the one driver for every
variant comparison (it replaces the single-use *_ab.py / *_time.py scripts of rounds 1-5).

    python tools/ab.py <leg> [--steps N] [--rounds R] [--settle MS] [--lib PATH] VARIANT ...

<leg>: a name of tools/pmc_drive.py's registry (the bench legs: dense_c48, mappm_c384_k10,
coarsen_1f, stepper_c96_r8, emulator_c384, ...).  VARIANT: ``name`` or
``name:ENV=V[,ENV2=V2...]``: the library's kernel-variant selectors (csrc/common.h
variant_env: FV3_DENSE_*, FV3_B3_*, FV3_MAPPM_*, FV3_COARSEN_*, FV3_EPILOGUE_PATH, ...),
set in this process with FV3_VARIANTS=1 and read by the library per launch.  Selectors
of variant kernels (other register targets, load distances, LDS scratch) act only on a
variants build: ``tools/build_variant.sh <name>`` then ``--lib tools/variants/lib<name>.so``
(the product library keeps the kernels its own heuristics pick).  Library builds are
compared by ``tools/ab.sh``.

Each round runs every variant in turn on the same workload (bench.timed_steps: clock settle,
warmup, N timed steps); prints mean ms per step (wall clock) and per launch (HIP events).
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def parse_variant(spec):
    name, _, env = spec.partition(":")
    pairs = {}
    for kv in filter(None, env.split(",")):
        k, _, v = kv.partition("=")
        pairs[k.strip()] = v.strip()
    return name, pairs


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("leg")
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--settle", type=float, default=150.0)
    ap.add_argument("--lib", default=None, help="library to load (FV3NET_AMD_LIB), e.g. a variants build")
    args = ap.parse_args(argv)
    if args.lib:
        os.environ["FV3NET_AMD_LIB"] = args.lib
    os.environ["FV3_VARIANTS"] = "1"
    import torch

    import bench
    from fv3net_amd import _native
    from pmc_drive import make

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    print(f"library: {_native.load().fv3_build_kind().decode()}  leg: {args.leg}", flush=True)
    variants = [parse_variant(v) for v in args.variants]
    touched = sorted({k for _, env in variants for k in env})
    wl = make(args.leg, dev)
    for rnd in range(args.rounds):
        for name, env in variants:
            for k in touched:
                os.environ.pop(k, None)
            os.environ.update(env)
            wall, launch = bench.timed_steps(wl.step, args.steps, 3, settle_ms=args.settle)
            print(f"round {rnd} {name:>16}: {wall / args.steps * 1e3:.4f} ms/step wall, "
                  f"{launch * 1e3:.4f} ms/launch", flush=True)
    for k in touched:
        os.environ.pop(k, None)


if __name__ == "__main__":
    main()
