"""Denoiser weights: data-only reader for the reference checkpoints + npz store.

The reference loads its denoisers with ``torch.load`` of whole pickled
``DataParallel(simple_CNN)`` objects (models/denoiser.py:18-21) or KAIR
state_dicts (models/network_dncnn.py:71).  Those files are *legacy* (non-zip)
torch serialisations.  We never unpickle them: ``read_legacy_checkpoint`` walks
the pickle opcode stream with ``pickletools.genops`` (a tokenizer) and a tiny
symbolic stack machine that only builds tuples/lists/dicts/strings/numbers and
records GLOBAL / REDUCE / BUILD as inert nodes.  Nothing from the file is
imported, called or executed.  Tensor bytes are then sliced out of the raw
storage section that follows the pickles.

Runtime (and the GPU box) only ever reads the converted ``weights/*.npz``
(plain float32 arrays, ``numpy.load(allow_pickle=False)``).

Layer order of ``simple_CNN`` (models/basic_models.py:15-18, forward :25-36):
``in_conv``, ``conv_list.0 .. conv_list.{depth-3}``, ``out_conv``; LeakyReLU
default slope 0.01 (:21), residual ``+ x_in`` (:36), clamps in/out
(models/denoiser.py:40,42).  KAIR ``DnCNN`` (network_dncnn.py:42-77):
``model.0``, ``model.2``, ..., ReLU, ``x - n``, no clamps.
"""
from __future__ import annotations

import io
import os
import pickletools
import struct
from collections import OrderedDict
from dataclasses import dataclass, field
from typing import List

import numpy as np

ACT_LEAKY_RELU = 0  # slope 0.01  (basic_models.py:21 -> nn.LeakyReLU())
ACT_RELU = 1        # KAIR 'R'    (network_dncnn.py:64-66)
LEAKY_SLOPE = 0.01

WEIGHTS_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "weights")


# --------------------------------------------------------------------------
# symbolic pickle walk (data only)
# --------------------------------------------------------------------------
@dataclass
class _Global:
    module: str
    name: str

    @property
    def qual(self) -> str:
        return f"{self.module}.{self.name}"


@dataclass
class _Node:
    """Result of REDUCE/NEWOBJ on a symbolic callable; nothing is called."""
    func: object
    args: tuple
    items: "OrderedDict" = field(default_factory=OrderedDict)  # SETITEM(S) targets
    appends: list = field(default_factory=list)
    state: object = None                                      # BUILD argument


@dataclass
class _PersId:
    pid: object


class _Mark:
    pass


_MARK = _Mark()


def _symbolic_load(ops):
    """Run the opcode stream of ONE pickle symbolically; returns the top object."""
    stack: list = []
    memo: dict = {}

    def pop_mark():
        items = []
        while True:
            v = stack.pop()
            if v is _MARK:
                break
            items.append(v)
        items.reverse()
        return items

    for op, arg, _pos in ops:
        name = op.name
        if name in ("PROTO", "FRAME"):
            continue
        if name == "STOP":
            return stack.pop()
        if name == "MARK":
            stack.append(_MARK)
        elif name in ("BININT", "BININT1", "BININT2", "LONG1", "LONG4", "INT", "LONG",
                      "BINFLOAT", "FLOAT", "BINUNICODE", "SHORT_BINUNICODE", "BINUNICODE8",
                      "UNICODE", "BINSTRING", "SHORT_BINSTRING", "STRING", "BINBYTES",
                      "SHORT_BINBYTES", "BINBYTES8"):
            stack.append(arg)
        elif name == "NONE":
            stack.append(None)
        elif name == "NEWTRUE":
            stack.append(True)
        elif name == "NEWFALSE":
            stack.append(False)
        elif name == "EMPTY_TUPLE":
            stack.append(())
        elif name == "TUPLE":
            stack.append(tuple(pop_mark()))
        elif name == "TUPLE1":
            stack.append((stack.pop(),))
        elif name == "TUPLE2":
            b = stack.pop(); a = stack.pop(); stack.append((a, b))
        elif name == "TUPLE3":
            c = stack.pop(); b = stack.pop(); a = stack.pop(); stack.append((a, b, c))
        elif name == "EMPTY_LIST":
            stack.append([])
        elif name == "LIST":
            stack.append(pop_mark())
        elif name == "APPEND":
            v = stack.pop(); tgt = stack[-1]
            (tgt.appends if isinstance(tgt, _Node) else tgt).append(v)
        elif name == "APPENDS":
            vs = pop_mark(); tgt = stack[-1]
            (tgt.appends if isinstance(tgt, _Node) else tgt).extend(vs)
        elif name == "EMPTY_DICT":
            stack.append(OrderedDict())
        elif name == "DICT":
            vs = pop_mark(); d = OrderedDict()
            for i in range(0, len(vs), 2):
                d[vs[i]] = vs[i + 1]
            stack.append(d)
        elif name == "SETITEM":
            v = stack.pop(); k = stack.pop(); tgt = stack[-1]
            (tgt.items if isinstance(tgt, _Node) else tgt)[k] = v
        elif name == "SETITEMS":
            vs = pop_mark(); tgt = stack[-1]
            d = tgt.items if isinstance(tgt, _Node) else tgt
            for i in range(0, len(vs), 2):
                d[vs[i]] = vs[i + 1]
        elif name == "GLOBAL":
            mod, _, nm = arg.partition(" ")
            stack.append(_Global(mod, nm))
        elif name == "STACK_GLOBAL":
            nm = stack.pop(); mod = stack.pop(); stack.append(_Global(mod, nm))
        elif name == "REDUCE":
            args = stack.pop(); fn = stack.pop(); stack.append(_Node(fn, tuple(args)))
        elif name == "NEWOBJ":
            args = stack.pop(); cls = stack.pop(); stack.append(_Node(cls, tuple(args)))
        elif name == "BUILD":
            st = stack.pop(); tgt = stack[-1]
            if isinstance(tgt, _Node):
                tgt.state = st
            # BUILD on a plain container is ignored (no behaviour to emulate)
        elif name == "BINPERSID":
            stack.append(_PersId(stack.pop()))
        elif name in ("BINPUT", "LONG_BINPUT", "PUT"):
            memo[arg] = stack[-1]
        elif name == "MEMOIZE":
            memo[len(memo)] = stack[-1]
        elif name in ("BINGET", "LONG_BINGET", "GET"):
            stack.append(memo[arg])
        elif name == "POP":
            stack.pop()
        elif name == "POP_MARK":
            pop_mark()
        elif name == "DUP":
            stack.append(stack[-1])
        elif name == "EMPTY_SET":
            stack.append(set())
        else:
            raise ValueError(f"unsupported pickle opcode {name} (file not a plain checkpoint?)")
    raise ValueError("pickle stream ended without STOP")


def _next_pickle(buf: io.BytesIO):
    """Tokenize one pickle from ``buf`` (advances past its STOP)."""
    ops = []
    for op, arg, pos in pickletools.genops(buf):
        ops.append((op, arg, pos))
        if op.name == "STOP":
            break
    return _symbolic_load(ops)


_DTYPES = {"FloatStorage": np.float32, "DoubleStorage": np.float64, "HalfStorage": np.float16,
           "LongStorage": np.int64, "IntStorage": np.int32}


def _tensor_spec(node):
    """_rebuild_parameter(_rebuild_tensor_v2(pid, off, size, stride, ...)) -> spec."""
    if isinstance(node, _Node) and isinstance(node.func, _Global):
        if node.func.name == "_rebuild_parameter":
            return _tensor_spec(node.args[0])
        if node.func.name == "_rebuild_tensor_v2":
            pid, offset, size, stride = node.args[0], node.args[1], node.args[2], node.args[3]
            assert isinstance(pid, _PersId)
            kind, stype, key = pid.pid[0], pid.pid[1], pid.pid[2]
            assert kind == "storage"
            return dict(key=str(key), dtype=_DTYPES[stype.name], offset=int(offset),
                        size=tuple(size), stride=tuple(stride))
    return None


def _walk_module(node, prefix, out):
    """Collect parameters of a symbolic nn.Module tree in registration order."""
    st = node.state
    if isinstance(st, tuple):
        st = st[0]
    if not isinstance(st, dict):
        return
    params = st.get("_parameters")
    if isinstance(params, _Node):
        params = params.items
    for k, v in (params or {}).items():
        spec = _tensor_spec(v)
        if spec is not None:
            out[prefix + k] = spec
    mods = st.get("_modules")
    if isinstance(mods, _Node):
        mods = mods.items
    for k, m in (mods or {}).items():
        if isinstance(m, _Node):
            _walk_module(m, prefix + k + ".", out)


def read_legacy_checkpoint(path: str) -> "OrderedDict[str, np.ndarray]":
    """Parameters of a legacy torch checkpoint, as float32 numpy arrays, in order."""
    raw = open(path, "rb").read()
    buf = io.BytesIO(raw)
    magic = _next_pickle(buf)
    if magic != 0x1950A86A20F9469CFC6C:
        raise ValueError(f"{path}: not a legacy torch checkpoint")
    _proto = _next_pickle(buf)
    _sysinfo = _next_pickle(buf)
    root = _next_pickle(buf)
    keys = _next_pickle(buf)
    specs: "OrderedDict[str, dict]" = OrderedDict()
    if isinstance(root, _Node) and isinstance(root.func, _Global) and root.func.name == "OrderedDict":
        for k, v in root.items.items():            # plain state_dict (KAIR)
            spec = _tensor_spec(v)
            if spec is not None:
                specs[k] = spec
    elif isinstance(root, _Node):
        _walk_module(root, "", specs)               # whole pickled module
    else:
        raise ValueError(f"{path}: unrecognised checkpoint root")
    # raw storages follow, in the order of `keys`: int64 numel + data
    pos = buf.tell()
    storages = {}
    dtype_of = {s["key"]: s["dtype"] for s in specs.values()}
    for key in keys:
        (numel,) = struct.unpack_from("<q", raw, pos)
        pos += 8
        dt = np.dtype(dtype_of.get(str(key), np.float32))
        storages[str(key)] = np.frombuffer(raw, dtype=dt, count=numel, offset=pos)
        pos += numel * dt.itemsize
    out: "OrderedDict[str, np.ndarray]" = OrderedDict()
    for name, s in specs.items():
        st = storages[s["key"]]
        n = int(np.prod(s["size"])) if s["size"] else 1
        el = st.itemsize
        arr = np.lib.stride_tricks.as_strided(st[s["offset"]:], shape=s["size"],
                                              strides=tuple(x * el for x in s["stride"]))
        assert arr.size == n
        out[name[len("module."):] if name.startswith("module.") else name] = \
            np.ascontiguousarray(arr, dtype=np.float32)
    return out


# --------------------------------------------------------------------------
# canonical layer list
# --------------------------------------------------------------------------
@dataclass
class DenoiserWeights:
    """Conv stack in forward order.  weights[i]: (cout, cin, 3, 3) f32, biases[i]: (cout,)."""
    channels: int
    weights: List[np.ndarray]
    biases: List[np.ndarray]
    act: int = ACT_LEAKY_RELU
    residual: int = +1      # +1: out = net(x) + x (simple_CNN); -1: out = x - net(x) (KAIR)
    clamp_io: int = 1       # clamp input and output to [0,1] (denoiser.py:40,42)
    name: str = ""

    @property
    def depth(self) -> int:
        return len(self.weights)

    @property
    def width(self) -> int:
        return int(self.weights[0].shape[0])

    def flat(self) -> np.ndarray:
        """[w0, b0, w1, b1, ...] concatenated (the C-ABI's pnp_set_denoiser layout)."""
        parts = []
        for w, b in zip(self.weights, self.biases):
            parts.append(np.ascontiguousarray(w, np.float32).ravel())
            parts.append(np.ascontiguousarray(b, np.float32).ravel())
        return np.concatenate(parts)

    def save_npz(self, path: str) -> None:
        arrs = {f"w{i:02d}": w for i, w in enumerate(self.weights)}
        arrs.update({f"b{i:02d}": b for i, b in enumerate(self.biases)})
        meta = np.array([self.channels, self.depth, self.act, self.residual, self.clamp_io], np.int64)
        np.savez(path, meta=meta, **arrs)

    @classmethod
    def load_npz(cls, path: str) -> "DenoiserWeights":
        with np.load(path, allow_pickle=False) as z:
            ch, depth, act, residual, clamp_io = (int(v) for v in z["meta"])
            ws = [np.asarray(z[f"w{i:02d}"], np.float32) for i in range(depth)]
            bs = [np.asarray(z[f"b{i:02d}"], np.float32) for i in range(depth)]
        return cls(ch, ws, bs, act, residual, clamp_io, os.path.basename(path))


def from_simple_cnn_state(sd, channels: int, name: str = "") -> DenoiserWeights:
    """simple_CNN parameter dict (basic_models.py:15-18 names) -> DenoiserWeights."""
    ws, bs = [sd["in_conv.weight"]], [sd["in_conv.bias"]]
    i = 0
    while f"conv_list.{i}.weight" in sd:
        ws.append(sd[f"conv_list.{i}.weight"]); bs.append(sd[f"conv_list.{i}.bias"]); i += 1
    ws.append(sd["out_conv.weight"]); bs.append(sd["out_conv.bias"])
    assert ws[0].shape[1] == channels and ws[-1].shape[0] == channels
    return DenoiserWeights(channels, ws, bs, ACT_LEAKY_RELU, +1, 1, name)


def from_kair_state(sd, channels: int, name: str = "") -> DenoiserWeights:
    """KAIR DnCNN state_dict ('model.{0,2,..}.weight', network_dncnn.py:60-68)."""
    idx = sorted({int(k.split(".")[1]) for k in sd if k.startswith("model.") and k.endswith(".weight")})
    ws = [sd[f"model.{j}.weight"] for j in idx]
    bs = [sd[f"model.{j}.bias"] for j in idx]
    assert ws[0].shape[1] == channels
    return DenoiserWeights(channels, ws, bs, ACT_RELU, -1, 0, name)


def convert_checkpoint(path: str, channels: int | None = None) -> DenoiserWeights:
    """Legacy .pth (either family) -> DenoiserWeights, data-only."""
    sd = read_legacy_checkpoint(path)
    name = os.path.splitext(os.path.basename(path))[0]
    if "in_conv.weight" in sd:
        ch = channels or int(sd["in_conv.weight"].shape[1])
        return from_simple_cnn_state(sd, ch, name)
    first = sd[next(iter(sd))]
    ch = channels or int(first.shape[1])
    return from_kair_state(sd, ch, name)


def resolve_weights(file_name: str, channels: int | None = None) -> DenoiserWeights:
    """Map the reference's ``path_prox`` (e.g. '.../nn/DnCNN_nobn_nch_3_nlev_0.01.pth')
    to the converted npz shipped in ``pnp-pds_amd/weights``; fall back to a data-only
    conversion if the .pth itself is present and no npz exists."""
    if file_name.endswith(".npz") and os.path.exists(file_name):
        return DenoiserWeights.load_npz(file_name)
    stem = os.path.basename(file_name)
    for ext in (".pth", ".npz", ".pt"):
        if stem.endswith(ext):
            stem = stem[: -len(ext)]
    npz = os.path.join(WEIGHTS_DIR, stem + ".npz")
    if os.path.exists(npz):
        w = DenoiserWeights.load_npz(npz)
    elif os.path.exists(file_name):
        w = convert_checkpoint(file_name, channels)
    else:
        raise FileNotFoundError(f"no converted weights for {file_name!r} (looked for {npz})")
    if channels is not None and w.channels != channels:
        raise ValueError(f"weights {stem} have {w.channels} channels, ch={channels} requested")
    return w


def random_weights(channels: int = 3, depth: int = 20, width: int = 64, seed: int = 0,
                   scale: float = 1.0) -> DenoiserWeights:
    """He-style random init of the simple_CNN architecture (for synthetic benches/tests)."""
    rng = np.random.default_rng(seed)
    ws, bs = [], []
    cin = channels
    for i in range(depth):
        cout = channels if i == depth - 1 else width
        std = scale * np.sqrt(2.0 / (cin * 9))
        ws.append((rng.standard_normal((cout, cin, 3, 3)) * std).astype(np.float32))
        bs.append((rng.standard_normal(cout) * 0.01).astype(np.float32))
        cin = cout
    return DenoiserWeights(channels, ws, bs, ACT_LEAKY_RELU, +1, 1, f"random{seed}")
