"""Generate golden vectors by IMPORTING THE REFERENCE (build container only).

    python tests/golden/make_golden.py [/root/reference]

The reference's hot path imports on CPU with four runtime shims and no
edits to /root/reference:
  1. ``bm3d`` (iteration.py:3, BM3D comparison methods only)  -> empty module
  2. ``skimage.metrics.structural_similarity`` (utils_eval.py:2) -> stub returning 0.0
     (SSIM is therefore *unpinned*)
  3. ``models.denoiser.load_checkpoint`` (denoiser.py:18-21) -> copies our converted npz
     weights (pnp-pds_amd/weights, produced by the data-only reader) into the reference's
     own ``simple_CNN``; the legacy pickle is never unpickled
  4. ``torch.cuda.synchronize`` (iteration.py:192) -> no-op (no GPU here)
Everything else — operators.py, models/basic_models.py, algorithm/admm.py,
iteration.test_iter, utils/utils_noise.py — runs as shipped.

Outputs (inputs + expected outputs, nothing else) go to tests/golden/*.npz.
"""
import os
import sys
import time
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.abspath(os.path.join(HERE, "..", ".."))
sys.path.insert(0, os.path.join(REPO, "pnp-pds_amd"))
from pnppds.weights import DenoiserWeights, WEIGHTS_DIR  # noqa: E402


def synthetic_image(C, H, W, seed):
    """Deterministic structured test image in [0,1]: gradients, sinusoids, rectangles."""
    rng = np.random.RandomState(seed)
    yy, xx = np.meshgrid(np.linspace(0, 1, H), np.linspace(0, 1, W), indexing="ij")
    img = np.zeros((C, H, W), np.float64)
    for c in range(C):
        f1, f2, ph = rng.uniform(1, 6), rng.uniform(1, 6), rng.uniform(0, 6.28)
        img[c] = 0.45 + 0.25 * np.sin(2 * np.pi * f1 * xx + ph) * np.cos(2 * np.pi * f2 * yy) + 0.2 * (xx - 0.5)
        for _ in range(4):
            y0, x0 = rng.randint(0, H - H // 4), rng.randint(0, W - W // 4)
            img[c, y0:y0 + rng.randint(4, H // 4), x0:x0 + rng.randint(4, W // 4)] += rng.uniform(-0.3, 0.3)
    return np.clip(img, 0, 1).astype(np.float32)


def install_shims(ref_root):
    sys.modules["bm3d"] = types.ModuleType("bm3d")
    sk = types.ModuleType("skimage")
    skm = types.ModuleType("skimage.metrics")
    skm.structural_similarity = lambda **kw: 0.0
    sk.metrics = skm
    sys.modules["skimage"] = sk
    sys.modules["skimage.metrics"] = skm
    sys.path.insert(0, ref_root)
    import torch
    torch.cuda.synchronize = lambda *a, **k: None
    import models.denoiser as md

    def load_checkpoint(model, file_name):
        stem = os.path.splitext(os.path.basename(file_name))[0]
        w = DenoiserWeights.load_npz(os.path.join(WEIGHTS_DIR, stem + ".npz"))
        sd = {"in_conv.weight": w.weights[0], "in_conv.bias": w.biases[0],
              "out_conv.weight": w.weights[-1], "out_conv.bias": w.biases[-1]}
        for i in range(1, w.depth - 1):
            sd[f"conv_list.{i-1}.weight"] = w.weights[i]
            sd[f"conv_list.{i-1}.bias"] = w.biases[i]
        model.module.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
        return model

    md.load_checkpoint = load_checkpoint


def degrade(x_true, phi, Id, deg_op, gaussian_nl, sp_nl, poisson_noise, poisson_alpha):
    """main.py:49-64 verbatim semantics, using the reference's own utils_noise."""
    from utils.utils_noise import add_gaussian_noise, add_salt_and_pepper_noise, apply_poisson_noise
    obs = phi(x_true)
    obs = add_gaussian_noise(obs, gaussian_nl, Id if deg_op in ("blur", "Id") else phi)
    if poisson_noise:
        obs = apply_poisson_noise(obs, poisson_alpha)
    obs = add_salt_and_pepper_noise(obs, sp_nl, Id if deg_op in ("blur", "Id") else phi)
    x0 = np.copy(obs)
    if poisson_noise:
        x0 = x0 / poisson_alpha
    return obs, x0


def main(ref_root="/root/reference"):
    install_shims(ref_root)
    import torch
    import operators as op
    import iteration
    from models.denoiser import Denoiser
    from models.network_dncnn import DnCNN
    from utils.utils_eval import eval_psnr

    path_kernel = os.path.join(ref_root, "blur_models", "blur_1.mat")
    nn_dir = os.path.join(ref_root, "nn")
    h = __import__("scipy.io").io.loadmat(path_kernel)["blur"]
    rng = np.random.default_rng(20261015)
    out = {}

    # ---- G1: observation operators -------------------------------------------------
    ops = {"h": h}
    for tag, shape in (("rgb64", (3, 64, 64)), ("gray64", (64, 64)), ("gray256", (256, 256)), ("rgb48x80", (3, 48, 80))):
        x = rng.standard_normal(shape)
        ops[f"x_{tag}"] = x
        for kind, rr in (("blur", 0.8), ("random_sampling", 0.8), ("random_sampling", 0.5)):
            if kind == "random_sampling" and (tag == "gray256" or (len(shape) == 3 and shape[0] != 3)):
                continue
            phi, adj = op.get_observation_operators(kind, path_kernel, rr)
            key = kind if kind == "blur" else f"rs{int(rr*10)}"
            ops[f"phi_{key}_{tag}"] = phi(x)
            ops[f"adj_{key}_{tag}"] = adj(x)
    # ---- G2: proximal operators ----------------------------------------------------------
    v = rng.standard_normal((3, 64, 64)) * 0.1
    x0 = rng.uniform(0, 1, (3, 64, 64))
    ops["prox_v"], ops["prox_x0"] = v, x0
    for nl, a in ((0.01, 0.95), (10.0, 1.0)):     # outside / inside the ball
        ops[f"l2_{nl}_{a}"] = op.proj_l2_ball(x0 + v, a, nl, 0.1, x0, 0.8)
    for sp in (0.0, 0.01, 0.1, 0.5):
        ops[f"l1_{sp}"] = op.proj_l1_ball(v, 0.95, sp, 0.8)
    ops["l1_inside"] = op.proj_l1_ball(v * 1e-4, 0.95, 0.1, 1)
    ops["gkl"] = op.prox_GKL(v * 10, 0.5, 300.0, np.round(x0 * 300))
    ops["psnr"] = np.array([eval_psnr(x0, x0 + v)])
    np.savez_compressed(os.path.join(HERE, "ops.npz"), **ops)
    print("ops.npz", len(ops))

    # ---- G3: denoisers --------------------------------------------------------------
    den = {}
    for ch, name in ((3, "DnCNN_nobn_nch_3_nlev_0.01"), (1, "DnCNN_nobn_nch_1_nlev_0.01")):
        d = Denoiser(os.path.join(nn_dir, name + ".pth"), ch)
        clean = synthetic_image(ch, 64, 64, seed=ch)
        xin = (clean + 0.03 * rng.standard_normal(clean.shape)).astype(np.float32)
        xin[:, :4, :4] = -0.2          # exercise the input clamp (denoiser.py:40)
        xin[:, -4:, -4:] = 1.3
        if ch == 1:
            xin = xin[0]
        den[f"in_{name}"] = xin
        den[f"out_{name}"] = d.denoise(xin)
    for ch, name, nb in ((3, "dncnn_color_blind", 20), (1, "dncnn_15", 17)):
        net = DnCNN(in_nc=ch, out_nc=ch, nc=64, nb=nb, act_mode="R", model_path=os.path.join(nn_dir, name + ".pth"))
        xin = synthetic_image(ch, 64, 64, seed=10 + ch) + 0.05 * rng.standard_normal((ch, 64, 64)).astype(np.float32)
        with torch.no_grad():
            o = net(torch.from_numpy(xin.astype(np.float32)).unsqueeze(0))[0].numpy()
        den[f"in_{name}"], den[f"out_{name}"] = xin.astype(np.float32), o
    np.savez_compressed(os.path.join(HERE, "denoiser.npz"), **den)
    print("denoiser.npz", len(den))

    # ---- G4 / G6: test_iter trajectories ------------------------------------------------
    cases = [
        # name,      method,        deg_op,            ch, sigma, sp_nl, poisson, g1,     g2,          a_n,  a_s,  lam, r,   iters, m1, m2
        ("A_blur",   "A-Proposed",  "blur",            3, 0.01, 0.0, False, 0.99,   0.99,        0.95, 1.0,  1.0, 0.8, 5, 15, 15),
        ("A_id",     "A-Proposed",  "Id",              3, 0.01, 0.0, False, 0.99,   0.99,        0.95, 1.0,  1.0, 0.8, 5, 15, 15),
        ("A_rs",     "A-Proposed",  "random_sampling", 3, 0.01, 0.0, False, 0.99,   0.99,        0.95, 1.0,  1.0, 0.8, 5, 15, 15),
        ("A_gray",   "A-Proposed",  "Id",              1, 0.01, 0.0, False, 0.99,   0.99,        0.95, 1.0,  1.0, 0.8, 5, 15, 15),
        ("B_blur",   "B-Proposed",  "blur",            3, 0.01, 0.1, False, 1.0,    0.49,        0.95, 0.95, 1.0, 0.8, 5, 15, 15),
        ("C_rs",     "C-Proposed",  "random_sampling", 3, 0.0,  0.0, True,  0.00035, 1 / 0.00035, 1.0, 1.0,  1.0, 0.5, 5, 15, 15),
        ("C_blur",   "C-Proposed",  "blur",            3, 0.0,  0.0, True,  0.00055, 1786.0,      1.0, 1.0,  1.0, 0.8, 5, 15, 15),
        ("ADMM_B2",  "comparisonB-2", "blur",          3, 0.01, 0.1, False, 0.99,   0.99,        0.95, 0.95, 1.0, 0.8, 1, 2, 2),
    ]
    for (name, method, deg, ch, sig, sp, pois, g1, g2, an, as_, lam, r, iters, m1, m2) in cases:
        phi, adj = op.get_observation_operators(deg, path_kernel, r)
        Id, _ = op.get_observation_operators("Id", path_kernel, r)
        xt = synthetic_image(ch, 64, 64, seed=100 + len(name))
        if ch == 1:
            xt = xt[0]
        obs, x0 = degrade(xt, phi, Id, deg, sig, sp, pois, 300)
        arch = f"DnCNN_nobn_nch_{ch}_nlev_0.01"
        t = time.perf_counter()
        res = iteration.test_iter(x0, obs, xt, phi, adj, g1, g2, as_, an, lam, m1, m2, 0.1, sig, sp, 300,
                                  os.path.join(nn_dir, arch + ".pth"), iters, method, ch, r)
        xs, ss, c, ps, _ssim, _t = res
        np.savez_compressed(os.path.join(HERE, f"iter_{name}.npz"), x_true=xt, x_obs=obs, x_0=x0,
                            x_out=xs, s_out=ss, c=c, psnr=ps,
                            params=np.array([g1, g2, as_, an, lam, m1, m2, 0.1, sig, sp, 300, iters, ch, r]),
                            method=np.array(method), deg_op=np.array(deg), arch=np.array(arch))
        print(f"iter_{name}.npz  psnr {ps[0]:.3f} -> {ps[-1]:.3f}  ({time.perf_counter()-t:.1f}s)")

    make_long_256(ref_root)


def make_long_256(ref_root="/root/reference"):
    """G5: long run at 256^2 (pins the 0.01 dB target)."""
    install_shims(ref_root)
    import operators as op
    import iteration
    path_kernel = os.path.join(ref_root, "blur_models", "blur_1.mat")
    nn_dir = os.path.join(ref_root, "nn")
    phi, adj = op.get_observation_operators("blur", path_kernel, 0.8)
    Id, _ = op.get_observation_operators("Id", path_kernel, 0.8)
    xt = synthetic_image(3, 256, 256, seed=7)
    obs, x0 = degrade(xt, phi, Id, "blur", 0.01, 0.0, False, 300)
    t = time.perf_counter()
    res = iteration.test_iter(x0, obs, xt, phi, adj, 0.99, 0.99, 1.0, 0.95, 1.0, 15, 15, 0.1, 0.01, 0.0, 300,
                              os.path.join(nn_dir, "DnCNN_nobn_nch_3_nlev_0.01.pth"), 120, "A-Proposed", 3, 0.8)
    np.savez_compressed(os.path.join(HERE, "long_A_blur_256.npz"), x_true=xt, x_obs=obs.astype(np.float32),
                        x_out=res[0].astype(np.float32), c=res[2], psnr=res[3])
    print(f"long_A_blur_256.npz psnr {res[3][0]:.3f} -> {res[3][-1]:.3f} ({time.perf_counter()-t:.1f}s)")


def make_driver_golden(ref_root="/root/reference"):
    """utils_textfile.py / utils_parse_args.py / utils_method_master.py outputs for fixed inputs
    (tests/golden/driver.json): the CSV text of a synthetic ``datas`` dict and the argument
    defaults, produced by the reference's own functions."""
    import json
    sys.path.insert(0, ref_root)
    from utils import utils_textfile as tf
    from utils import utils_parse_args as pa
    from utils.utils_method_master import get_algorithm_denoiser
    results = {i: {"filename": f"{i:02d}.png", "PSNR": 20.0 + i / 3, "SSIM": 0.5 + i / 7,
                   "PSNR_observation": 15.0 + i / 9, "SSIM_observation": 0.25 + i / 11} for i in range(3)}
    datas = {"experimental_settings": pa.parse_args_exp({"gaussian_nl": 0.01, "deg_op": "random_sampling"}),
             "method": pa.parse_args_method({"method": "A-Proposed", "gamma1": 0.99, "alpha_n": 0.94}),
             "configs": pa.parse_args_configs({}), "results": results}
    from utils.utils_unparse_args import unparse_args_configs, unparse_args_exp, unparse_args_method
    datas["experimental_settings"] = unparse_args_exp(*datas["experimental_settings"])
    datas["method"] = unparse_args_method(*datas["method"])
    datas["configs"] = unparse_args_configs(*datas["configs"])
    alg, den = get_algorithm_denoiser("A-Proposed")
    datas["summary"] = {"algorithm": alg, "denoiser": den, "Average_PSNR": 21.0, "Average_SSIM": 0.6}
    out = {"datas": {k: v for k, v in datas.items() if k != "results"},
           "results": [results[i] for i in range(3)],
           "header": tf.get_csv_header(), "data": tf.get_csv_data(datas), "footer": tf.get_csv_footer(datas),
           "defaults": {"exp": list(pa.parse_args_exp({})), "method": list(pa.parse_args_method({})),
                        "configs": list(pa.parse_args_configs({}))},
           "methods": {m: list(get_algorithm_denoiser(m)) for m in
                       ("A-Proposed", "A-PDS-TV", "C-RED-DnCNN", "comparisonB-2", "nope")}}
    with open(os.path.join(HERE, "driver.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("driver.json")


CMP_CASES = [
    # name,        method,                   deg_op, ch, sigma, sp,  pois,  g1,      g2,          a_n,  a_s,  lam, r,   iters, m1, m2, arch
    ("A_pnpfbs",  "A-PnPFBS-DnCNN",          "blur", 3, 0.01, 0.0, False, 1.0,     0.99,        0.95, 0.95, 1.99, 1.0, 4, 15, 15, None),
    ("A_pdstv",   "A-PDS-TV",                "blur", 3, 0.01, 0.0, False, 0.125,   0.99,        0.9,  0.95, 1.0, 1.0, 6, 15, 15, None),
    ("A_fbstv",   "A-FBS-TV",                "random_sampling", 3, 0.01, 0.0, False, 0.1, 0.99,  0.9,  0.95, 1.0, 0.8, 6, 15, 15, None),
    ("A_red",     "A-RED-DnCNN",             "blur", 3, 0.01, 0.0, False, 1.0,     0.99,        0.95, 0.95, 0.4, 1.0, 4, 15, 15, None),
    ("A_unstable", "A-PnPPDS-unstable-DnCNN", "blur", 3, 0.01, 0.0, False, 0.99,   0.99,        0.95, 0.95, 1.0, 1.0, 4, 15, 15,
     "dncnn_color_blind"),
    ("B3_htv",    "comparisonB-3",           "blur", 3, 0.01, 0.1, False, 0.1,     0.99,        0.95, 0.95, 1.0, 1.0, 6, 15, 15, None),
    ("C_admm",    "C-PnPADMM-DnCNN",         "blur", 3, 0.0,  0.0, True,  0.99,    0.99,        0.95, 0.95, 1.0, 1.0, 3, 5, 3, None),
    ("C_red",     "C-RED-DnCNN",             "random_sampling", 3, 0.0, 0.0, True, 1.0, 0.99,    0.95, 0.95, 0.5, 0.5, 3, 5, 2, None),
    ("C_unstable", "C-PnP-unstable-DnCNN",   "random_sampling", 1, 0.0, 0.0, True, 0.00035, 1 / 0.00035, 1.0, 1.0, 1.0, 0.5, 4, 15, 15,
     "dncnn_15"),
]


def make_cmp_golden(ref_root="/root/reference"):
    """Trajectories of the comparison methods (iteration.py:71-180, BM3D excluded).
    comparisonB-4 / -5 are absent: the reference raises UnboundLocalError for them
    (denoiser_J is only built for names containing 'Proposed' or 'DnCNN', iteration.py:40-41)."""
    install_shims(ref_root)
    import operators as op
    import iteration
    path_kernel = os.path.join(ref_root, "blur_models", "blur_1.mat")
    nn_dir = os.path.join(ref_root, "nn")
    for (name, method, deg, ch, sig, sp, pois, g1, g2, an, as_, lam, r, iters, m1, m2, arch) in CMP_CASES:
        phi, adj = op.get_observation_operators(deg, path_kernel, r)
        Id, _ = op.get_observation_operators("Id", path_kernel, r)
        xt = synthetic_image(ch, 64, 64, seed=300 + len(name))
        if ch == 1:
            xt = xt[0]
        obs, x0 = degrade(xt, phi, Id, deg, sig, sp, pois, 300)
        arch = arch or f"DnCNN_nobn_nch_{ch}_nlev_0.01"
        gad = 0.1
        t = time.perf_counter()
        res = iteration.test_iter(x0, obs, xt, phi, adj, g1, g2, as_, an, lam, m1, m2, gad, sig, sp, 300,
                                  os.path.join(nn_dir, arch + ".pth"), iters, method, ch, r)
        xs, ss, c, ps, _ssim, _t = res
        np.savez_compressed(os.path.join(HERE, f"iter_cmp_{name}.npz"), x_true=xt, x_obs=obs, x_0=x0,
                            x_out=np.asarray(xs), s_out=ss, c=c, psnr=ps,
                            params=np.array([g1, g2, as_, an, lam, m1, m2, gad, sig, sp, 300, iters, ch, r]),
                            method=np.array(method), deg_op=np.array(deg), arch=np.array(arch))
        print(f"iter_cmp_{name}.npz  psnr {ps[0]:.3f} -> {ps[-1]:.3f}  ({time.perf_counter()-t:.1f}s)")


LONG_CASES = [
    # name,          method,       deg_op,            ch, size, sigma, sp,  pois,  g1,      g2,          a_n,  a_s,  lam, r,   iters
    ("A_blur_1200",  "A-Proposed", "blur",            3, 256, 0.01, 0.0, False, 0.99,    0.99,        0.95, 1.0,  1.0, 0.8, 1200),
    ("B_blur_300",   "B-Proposed", "blur",            3, 128, 0.01, 0.1, False, 1.0,     0.49,        0.95, 0.95, 1.0, 0.8, 300),
    ("C_rs_300",     "C-Proposed", "random_sampling", 3, 128, 0.0,  0.0, True,  0.00035, 1 / 0.00035, 1.0,  1.0,  1.0, 0.5, 300),
    # random-sampling experiments run 3000 iterations (main.py:136-139)
    ("C_rs_3000",    "C-Proposed", "random_sampling", 3, 128, 0.0,  0.0, True,  0.00035, 1 / 0.00035, 1.0,  1.0,  1.0, 0.5, 3000),
    # round 3: the regimes of main.py:130-139 beyond sigma = 0.01 blur (VERDICT r02 "missing" 1)
    # BASELINE config 1 at full size: gray 256^2, Id (PSNR 45-50 dB, where fp16 weights cost 0.07 dB)
    ("A_gray_id_1200", "A-Proposed", "Id",            1, 256, 0.01, 0.0, False, 0.99,    0.99,        0.95, 1.0,  1.0, 0.8, 1200),
    # the random-sampling experiment: 3000 iterations (main.py:136-139), r = 0.8
    ("A_rs_3000",    "A-Proposed", "random_sampling", 3, 128, 0.01, 0.0, False, 0.99,    0.99,        0.95, 1.0,  1.0, 0.8, 3000),
    # the lowest noise level of the grid (main.py:130), blur and random sampling
    ("A_blur_s0025_1200", "A-Proposed", "blur",       3, 128, 0.0025, 0.0, False, 0.99,  0.99,        0.95, 1.0,  1.0, 0.8, 1200),
    ("A_rs_s0025_3000", "A-Proposed", "random_sampling", 3, 128, 0.0025, 0.0, False, 0.99, 0.99,      0.95, 1.0,  1.0, 0.8, 3000),
    # comparisonB-2 (BASELINE config 5's method) at its config's inner counts m1 = 35, m2 = 5
    ("ADMM_B2_30",   "comparisonB-2", "blur",         3, 128, 0.01, 0.1, False, 0.99,    0.99,        0.95, 0.95, 1.0, 0.8, 30),
    # round 4: the fp16 regimes at the lengths they run
    # ours-B blur + salt-and-pepper for the blur experiments' 1200 iterations (main.py:136-137)
    ("B_blur_1200",  "B-Proposed", "blur",            3, 128, 0.01, 0.1, False, 1.0,     0.49,        0.95, 0.95, 1.0, 0.8, 1200),
    # comparisonB-2 at m1 = 35, m2 = 5 for 200 outer iterations (7 000 denoiser calls)
    ("ADMM_B2_200",  "comparisonB-2", "blur",         3, 128, 0.01, 0.1, False, 0.99,    0.99,        0.95, 0.95, 1.0, 0.8, 200),
    # the grid's lowest noise level with its largest ball, alpha_n = 0.8 + 10 * 0.02 (main.py:130,143)
    ("A_blur_s0025_a100_1200", "A-Proposed", "blur",  3, 128, 0.0025, 0.0, False, 0.99,  0.99,        1.0,  1.0,  1.0, 0.8, 1200),
    # the rest of main.py's blur grid for the fp16 policy: the other noise levels (:130), the
    # smallest ball alpha_n = 0.82 (:143), and the two DnCNN comparison methods the grid runs
    # (:133,148-152: gamma1 = 1, myLambda in 0.2 .. 1.99)
    ("A_blur_s0005_1200", "A-Proposed", "blur",       3, 128, 0.005, 0.0, False, 0.99,   0.99,        0.95, 1.0,  1.0, 0.8, 1200),
    ("A_blur_s002_1200", "A-Proposed", "blur",        3, 128, 0.02,  0.0, False, 0.99,   0.99,        0.95, 1.0,  1.0, 0.8, 1200),
    ("A_blur_s004_1200", "A-Proposed", "blur",        3, 128, 0.04,  0.0, False, 0.99,   0.99,        0.95, 1.0,  1.0, 0.8, 1200),
    ("A_blur_s0025_a082_1200", "A-Proposed", "blur",  3, 128, 0.0025, 0.0, False, 0.99,  0.99,        0.82, 1.0,  1.0, 0.8, 1200),
    ("FBS_blur_1200", "A-PnPFBS-DnCNN", "blur",       3, 128, 0.01,  0.0, False, 1.0,    0.99,        0.95, 1.0,  1.0, 0.8, 1200),
    ("FBS_blur_s0025_1200", "A-PnPFBS-DnCNN", "blur", 3, 128, 0.0025, 0.0, False, 1.0,   0.99,        0.95, 1.0,  1.0, 0.8, 1200),
    ("RED_blur_1200", "A-RED-DnCNN", "blur",          3, 128, 0.01,  0.0, False, 1.0,    0.99,        0.95, 1.0,  1.0, 0.8, 1200),
    ("RED_blur_s0025_1200", "A-RED-DnCNN", "blur",    3, 128, 0.0025, 0.0, False, 1.0,   0.99,        0.95, 1.0,  1.0, 0.8, 1200),
    # the grid's higher noise levels (main.py:130) for the other fp16-candidate methods: ours-A's
    # fp16 error grows with sigma (0.0055 / 0.0068 dB at 0.02 / 0.04), so the policy needs them too
    ("B_blur_s002_1200", "B-Proposed", "blur",        3, 128, 0.02, 0.1, False, 1.0,     0.49,        0.95, 0.95, 1.0, 0.8, 1200),
    ("B_blur_s004_1200", "B-Proposed", "blur",        3, 128, 0.04, 0.1, False, 1.0,     0.49,        0.95, 0.95, 1.0, 0.8, 1200),
    ("FBS_blur_s004_1200", "A-PnPFBS-DnCNN", "blur",  3, 128, 0.04,  0.0, False, 1.0,    0.99,        0.95, 1.0,  1.0, 0.8, 1200),
    ("RED_blur_s004_1200", "A-RED-DnCNN", "blur",     3, 128, 0.04,  0.0, False, 1.0,    0.99,        0.95, 1.0,  1.0, 0.8, 1200),
    ("ADMM_B2_s004_30", "comparisonB-2", "blur",      3, 128, 0.04, 0.1, False, 0.99,    0.99,        0.95, 0.95, 1.0, 0.8, 30),
    # round 5: comparisonB-2 above sigma 0.01, where auto runs fp16w2, at the 200
    # outer iterations (m1 = 35, m2 = 5) that qualified fp16 at sigma 0.01
    ("ADMM_B2_s002_200", "comparisonB-2", "blur",     3, 128, 0.02, 0.1, False, 0.99,    0.99,        0.95, 0.95, 1.0, 0.8, 200),
    ("ADMM_B2_s004_200", "comparisonB-2", "blur",     3, 128, 0.04, 0.1, False, 0.99,    0.99,        0.95, 0.95, 1.0, 0.8, 200),
]
LONG_INNER = {"ADMM_B2_30": (35, 5), "ADMM_B2_200": (35, 5), "ADMM_B2_s004_30": (35, 5),   # (m1, m2) if not 15, 15
              "ADMM_B2_s002_200": (35, 5), "ADMM_B2_s004_200": (35, 5)}


def make_long_golden(ref_root="/root/reference", only=None):
    """Long trajectories at the lengths the experiments run (main.py:136-139: 1200 iterations
    for blur), so the 0.01 dB PSNR bound is checked over every iteration rather than
    extrapolated from 120: ours-A 3x256^2 blur for 1200 iterations (the metric's method,
    operator and image size), ours-B blur + salt-and-pepper and ours-C random sampling + Poisson
    at 3x128^2 for 300.  Stored: inputs, the per-iteration c and PSNR, the final x in fp32
    (round 6: fp16 capped the x check at half an fp16 ulp, 2.4e-4)."""
    install_shims(ref_root)
    import operators as op
    import iteration
    path_kernel = os.path.join(ref_root, "blur_models", "blur_1.mat")
    nn_dir = os.path.join(ref_root, "nn")
    for (name, method, deg, ch, n, sig, sp, pois, g1, g2, an, as_, lam, r, iters) in LONG_CASES:
        if only and name not in only:
            continue
        phi, adj = op.get_observation_operators(deg, path_kernel, r)
        Id, _ = op.get_observation_operators("Id", path_kernel, r)
        xt = synthetic_image(ch, n, n, seed=7 if n == 256 else 500 + len(name))
        if ch == 1:
            xt = xt[0]                      # the reference's grayscale images are (H, W)
        obs, x0 = degrade(xt, phi, Id, deg, sig, sp, pois, 300)
        arch = f"DnCNN_nobn_nch_{ch}_nlev_0.01"
        m1, m2 = LONG_INNER.get(name, (15, 15))
        t = time.perf_counter()
        res = iteration.test_iter(x0, obs, xt, phi, adj, g1, g2, as_, an, lam, m1, m2, 0.1, sig, sp, 300,
                                  os.path.join(nn_dir, arch + ".pth"), iters, method, ch, r)
        xs, ss, c, ps, _ssim, _t = res
        small = (lambda a: np.asarray(a, np.float32)) if n >= 256 else np.asarray   # fixture size
        np.savez_compressed(os.path.join(HERE, f"long_{name}.npz"), x_true=xt, x_obs=small(obs),
                            x_0=small(x0), x_out=np.asarray(xs).astype(np.float32), c=c, psnr=ps,
                            params=np.array([g1, g2, as_, an, lam, m1, m2, 0.1, sig, sp, 300, iters, ch, r]),
                            method=np.array(method), deg_op=np.array(deg), arch=np.array(arch))
        print(f"long_{name}.npz psnr {ps[0]:.3f} -> {ps[-1]:.3f} ({time.perf_counter()-t:.1f}s)", flush=True)


def make_weights_pin(ref_root="/root/reference"):
    """Pin of the simple_CNN weight conversion (tests/golden/weights_pin.json): the reference
    loads a checkpoint with a strict load_state_dict into simple_CNN(depth=20)
    (models/denoiser.py:18-30), so the checkpoint's parameter names, order and shapes are the
    module's state_dict.  Recorded here: that state_dict (names + shapes, from the reference's
    own class), and per layer the SHA-256 of our data-only reader's arrays straight from the
    .pth; tests/test_weights_pin.py checks the shipped npz layers against both."""
    import hashlib
    import json
    sys.path.insert(0, ref_root)
    from models.basic_models import simple_CNN
    from pnppds.weights import read_legacy_checkpoint
    out = {}
    for ch, name in ((3, "DnCNN_nobn_nch_3_nlev_0.01"), (1, "DnCNN_nobn_nch_1_nlev_0.01"),
                     (1, "DnCNN_nobn_nch_1_nlev_0.009")):
        net = simple_CNN(n_ch_in=ch, n_ch_out=ch, n_ch=64, nl_type="relu", depth=20, bn=False)
        keys = [(k, list(v.shape)) for k, v in net.state_dict().items()]
        raw = read_legacy_checkpoint(os.path.join(ref_root, "nn", name + ".pth"))
        out[name] = {"module_state_dict": keys,
                     "reader_keys": list(raw.keys()),
                     "sha256": {k: hashlib.sha256(np.ascontiguousarray(v, np.float32).tobytes()).hexdigest()
                                for k, v in raw.items()}}
    with open(os.path.join(HERE, "weights_pin.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("weights_pin.json")


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--weights-pin":
        make_weights_pin(*sys.argv[2:])
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "--long256":
        make_long_256(*sys.argv[2:])
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "--long":
        make_long_golden(only=sys.argv[2:] or None)
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "--cmp":
        make_cmp_golden(*sys.argv[2:])
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "--driver":
        make_driver_golden(*sys.argv[2:])
    else:
        main(*sys.argv[1:])
