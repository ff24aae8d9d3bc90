"""One-time conversion of the reference's checkpoints (reference nn/*.pth) to npz.

Runs in the build container only (the reference does not exist on the GPU box).
Uses the data-only reader in pnppds.weights: no unpickling, nothing executed.

    python tools/convert_weights.py [/root/reference/nn]
"""
import glob
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "pnp-pds_amd"))

from pnppds.weights import WEIGHTS_DIR, convert_checkpoint  # noqa: E402


def main(src: str = "/root/reference/nn") -> None:
    os.makedirs(WEIGHTS_DIR, exist_ok=True)
    for path in sorted(glob.glob(os.path.join(src, "*.pth"))):
        w = convert_checkpoint(path)
        out = os.path.join(WEIGHTS_DIR, os.path.splitext(os.path.basename(path))[0] + ".npz")
        w.save_npz(out)
        n = sum(a.size for a in w.weights) + sum(b.size for b in w.biases)
        print(f"{os.path.basename(path)} -> {os.path.relpath(out)}  ch={w.channels} depth={w.depth} "
              f"act={'leaky' if w.act == 0 else 'relu'} residual={w.residual:+d} params={n}")


if __name__ == "__main__":
    main(*sys.argv[1:])
