"""The shipped simple_CNN weights (pnp-pds_amd/weights/*.npz) are the reference checkpoints'
parameters, layer for layer (CPU only).

The reference loads a checkpoint with a strict ``load_state_dict`` into
``simple_CNN(depth=20)`` (models/denoiser.py:18-30), so the checkpoint's parameters map to
the module's state_dict by name.  tests/golden/weights_pin.json (make_golden.py
--weights-pin) holds that state_dict's names and shapes, taken from the reference's own class,
and the SHA-256 of every array our data-only reader takes straight from the .pth.  Checked
here: the npz layer i is the state_dict entry i (shape), its bytes are the reader's array of
that name (hash), and — where the reference tree is present — the reader's names are the
module's names in the module's order.
"""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN
from pnppds.weights import WEIGHTS_DIR, DenoiserWeights, read_legacy_checkpoint

PIN = json.load(open(os.path.join(GOLDEN, "weights_pin.json")))
REF_NN = "/root/reference/nn"


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a, np.float32).tobytes()).hexdigest()


@pytest.mark.parametrize("name", sorted(PIN))
def test_npz_layers_are_the_module_state_dict(name):
    pin = PIN[name]
    w = DenoiserWeights.load_npz(os.path.join(WEIGHTS_DIR, name + ".npz"))
    flat = []
    for wi, bi in zip(w.weights, w.biases):
        flat += [wi, bi]
    keys = pin["module_state_dict"]
    assert len(flat) == len(keys) == 40                       # depth 20: weight + bias per layer
    for arr, (key, shape) in zip(flat, keys):
        assert list(arr.shape) == shape, (key, arr.shape, shape)
        assert sha(arr) == pin["sha256"][key], key            # the reader's array of that name


@pytest.mark.skipif(not os.path.isdir(REF_NN), reason="reference checkpoints not present")
@pytest.mark.parametrize("name", sorted(PIN))
def test_reader_names_follow_the_module(name):
    raw = read_legacy_checkpoint(os.path.join(REF_NN, name + ".pth"))
    assert list(raw.keys()) == [k for k, _ in PIN[name]["module_state_dict"]]
    for k, v in raw.items():
        assert sha(v) == PIN[name]["sha256"][k]
