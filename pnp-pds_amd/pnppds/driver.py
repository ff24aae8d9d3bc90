"""Experiment driver and results format of the reference.

    main.py:16-101     test_all_images(experimental_settings_arg, method_arg, configs_arg)
    main.py:103-123    main(): parameter sweep, one CSV line per experiment
    utils/utils_parse_args.py / utils_unparse_args.py   argument defaults
    utils/utils_method_master.py                        get_algorithm_denoiser
    utils/utils_textfile.py                             SUMMARY CSV
    utils/utils_image.py                                save_imgs

Same arguments, defaults, result dictionary (``datas`` with experimental_settings / method /
configs / results / summary) and CSV text.  Differences, all at the file boundary:

* Images of the same shape are solved together as one batch on the device (the reference
  loops over them one by one); every image still gets main.py's reseeded noise, so the
  per-image results are the ones test_iter gives for that image alone.
* Images are read with PIL (cv2 is not in this image): ``read_image`` returns cv2.imread's
  BGR channel order scaled to [0,1] float32, and gray uses cv2's BGR2GRAY weights
  (0.299 R + 0.587 G + 0.114 B in float32; OpenCV's summation order is not pinned).
* Output paths use os.path.join and os.path.basename (the reference hard-codes Windows
  ``\\`` separators, main.py:75,82,120); ``CPU_time`` is the device wall time per iteration
  and image (batch time / batch size).
* ``result_output`` saves the PSNR curve as a PNG next to the images instead of plt.show().
"""
from __future__ import annotations

import datetime
import glob
import os

import numpy as np

DEFAULT_CONFIG = {"root_folder": "./", "path_test": "./img/test/", "path_result": "./result/",
                  "pattern_red": "*.png"}

METHOD_TABLE = {   # utils_method_master.py:4-20
    "A-Proposed": ("PnP-PDS", "DnCNN"),
    "A-PnPFBS-DnCNN": ("PnP-FBS", "DnCNN"),
    "A-PnPPDS-BM3D": ("PnP-PDS", "BM3D"),
    "A-PnPFBS-BM3D": ("PnP-FBS", "BM3D"),
    "A-PDS-TV": ("PDS", ""),
    "A-RED-DnCNN": ("RED-SD", "DnCNN"),
    "A-PnPPDS-unstable-DnCNN": ("PnP-PDS", "DnCNN (unstable)"),
    "B-Proposed": ("PnP-PDS", "DnCNN"),
    "C-Proposed": ("PnP-PDS", "DnCNN"),
    "C-PnPPDS-BM3D": ("PnP-PDS", "BM3D"),
    "C-PnPADMM-DnCNN": ("PnP-ADMM", "DnCNN"),
    "C-RED-DnCNN": ("RED-ADMM", "DnCNN"),
    "C-PnP-unstable-DnCNN": ("PnP-PDS", "DnCNN (unstable)"),
}


# ---- utils_parse_args.py / utils_unparse_args.py -----------------------------------------------
def parse_args_exp(args):
    return (args.get("gaussian_nl", 0), args.get("sp_nl", 0), args.get("poisson_noise", False),
            args.get("poisson_alpha", 300), args.get("deg_op", "blur"), args.get("r", 0.8))


def parse_args_method(args):
    return (args.get("method", "ours-A"), args.get("architecture", "DnCNN_nobn_nch_3_nlev_0.01"),
            args.get("max_iter", 10), args.get("gamma1", 1), args.get("gamma2", 1), args.get("alpha_n", 1),
            args.get("alpha_s", 1), args.get("myLambda", 1), args.get("m1", 15), args.get("m2", 15),
            args.get("gammaInADMMStep1", 0.1))


def parse_args_configs(args):
    return args.get("ch", 3), args.get("add_timestamp", True), args.get("result_output", False)


def unparse_args_exp(gaussian_nl, sp_nl, poisson_noise, poisson_alpha, deg_op, r):
    return {"gaussian_nl": gaussian_nl, "sp_nl": sp_nl, "poisson_noise": poisson_noise,
            "poisson_alpha": poisson_alpha, "deg_op": deg_op, "r": r}


def unparse_args_method(method, architecture, max_iter, gamma1, gamma2, alpha_n, alpha_s, myLambda, m1, m2,
                        gammaInADMMStep1):
    return {"method": method, "architecture": architecture, "max_iter": max_iter, "gamma1": gamma1,
            "gamma2": gamma2, "alpha_n": alpha_n, "alpha_s": alpha_s, "myLambda": myLambda, "m1": m1, "m2": m2,
            "gammaInADMMStep1": gammaInADMMStep1}


def unparse_args_configs(ch, add_timestamp, result_output):
    return {"ch": ch, "add_timestamp": add_timestamp, "result_output": result_output}


def get_algorithm_denoiser(method):
    return METHOD_TABLE.get(method, ("unknown algorithm", "unknown denoiser"))


# ---- image files (cv2.imread / utils_image.save_img semantics) ---------------------------------
def read_image(path, ch):
    """main.py:41-48: float32/255 in cv2's BGR order -> (3,H,W), or BGR2GRAY -> (H,W)."""
    from PIL import Image
    rgb = np.asarray(Image.open(path).convert("RGB"), dtype=np.float32) / np.float32(255.0)
    bgr = rgb[..., ::-1]
    if ch == 1:
        return (np.float32(0.114) * bgr[..., 0] + np.float32(0.587) * bgr[..., 1]
                + np.float32(0.299) * bgr[..., 2]).astype(np.float32)
    return np.ascontiguousarray(np.moveaxis(bgr, -1, 0))


def save_img(picture, path_picture, format=".png"):
    """utils_image.py:4-12: clip to [0,1], uint8(x*255) (truncation), BGR planes."""
    from PIL import Image
    p = np.array(picture, dtype=np.float64)
    if p.ndim == 3:
        p = np.moveaxis(p, 0, 2)[..., ::-1]        # BGR (C,H,W) -> RGB (H,W,C) for PIL
    p[p > 1.0] = 1.0
    p[p < 0.0] = 0.0
    Image.fromarray(np.uint8(p * 255.0)).save(path_picture + format)


def save_imgs(pictures, path_pictures, format=".png"):
    for pic, path in zip(pictures, path_pictures):
        save_img(pic, path, format)


# ---- utils_textfile.py ----------------------------------------------------------------------
def get_csv_header():
    return ("Observation,Gaussian_noise,Poisson_alpha,method,algorithm,denoiser,PSNR,SSIM,gamma1,gamma2,"
            "alpha_n,myLambda,max_iter,m1,m2,r,ch,"
            "Result PSNR - Result SSIM - Observed PSNR - Observed SSIM (for each images)\n")


def get_csv_data(data):
    e, m, s, c = data["experimental_settings"], data["method"], data["summary"], data["configs"]
    fields = [e["deg_op"], e["gaussian_nl"], e["poisson_alpha"], m["method"], s["algorithm"], s["denoiser"],
              s["Average_PSNR"], s["Average_SSIM"], m["gamma1"], m["gamma2"], m["alpha_n"], m["myLambda"],
              m["max_iter"], m["m1"], m["m2"], e["r"], c["ch"]]
    out = "".join(str(f) + "," for f in fields)
    for key in ("PSNR", "SSIM", "PSNR_observation", "SSIM_observation"):
        out += "".join(str(r[key]) + "," for r in data["results"].values())
    return out


def get_csv_footer(data):
    return "".join(str(r["filename"]) + "," for r in data["results"].values())


def touch_textfile(filepath):
    with open(filepath, "w") as f:
        f.write(get_csv_header())


def write_textfile(filepath, data):
    with open(filepath, "a") as f:
        f.write(get_csv_data(data) + "\n")


def add_footer_textfile(filepath, data):
    with open(filepath, "a") as f:
        f.write(get_csv_footer(data) + "\n")


# ---- main.py:16-101 ---------------------------------------------------------------------------
def _eval_psnr_ssim(ctx, x_true, x):
    """utils_eval.eval_psnr / eval_ssim on the device for one image ((C,H,W) or (H,W))."""
    import torch
    t = np.asarray(x_true, np.float32)
    v = np.asarray(x, np.float32)
    shp = (1, 1) + t.shape if t.ndim == 2 else (1,) + t.shape
    dt = torch.from_numpy(np.ascontiguousarray(t.reshape(shp))).to(f"cuda:{ctx.device}")
    dv = torch.from_numpy(np.ascontiguousarray(v.reshape(shp))).to(f"cuda:{ctx.device}")
    torch.cuda.synchronize(dt.device)
    psnr = float(ctx.op_psnr(dt.data_ptr(), dv.data_ptr(), 1, t.size)[0])
    ssim = float(ctx.op_ssim(dt.data_ptr(), dv.data_ptr(), 1, *shp[1:])[0])
    return psnr, ssim


def test_all_images(experimental_settings_arg=None, method_arg=None, configs_arg=None, config=None,
                    max_batch=64, save_images=True, save_data=True, verbose=True):
    """main.py:16-101 on the device.  Returns ``datas`` in the reference's layout."""
    from ._device import get_ctx
    from .iteration import test_iter_batch
    from .noise import make_observation_batch
    from .operators import get_observation_operators

    cfg = dict(DEFAULT_CONFIG, **(config or {}))
    gaussian_nl, sp_nl, poisson_noise, poisson_alpha, deg_op, r = parse_args_exp(experimental_settings_arg or {})
    (method, architecture, max_iter, gamma1, gamma2, alpha_n, alpha_s, myLambda, m1, m2,
     gammaInADMMStep1) = parse_args_method(method_arg or {})
    ch, add_timestamp, result_output = parse_args_configs(configs_arg or {})
    experimental_settings_all = unparse_args_exp(gaussian_nl, sp_nl, poisson_noise, poisson_alpha, deg_op, r)
    method_all = unparse_args_method(method, architecture, max_iter, gamma1, gamma2, alpha_n, alpha_s, myLambda,
                                     m1, m2, gammaInADMMStep1)
    configs_all = unparse_args_configs(ch, add_timestamp, result_output)

    path_result = cfg["path_result"]
    path_kernel = os.path.join(cfg["root_folder"], "blur_models", "blur_1.mat")
    path_prox = os.path.join(cfg["root_folder"], "nn", architecture + ".pth")
    path_images = sorted(glob.glob(os.path.join(cfg["path_test"], cfg["pattern_red"])))
    n_img = len(path_images)
    psnr, ssim, cpu_time = np.zeros(n_img), np.zeros(n_img), np.zeros(n_img)
    results = {}
    if save_images or save_data:
        os.makedirs(path_result, exist_ok=True)

    ctx = get_ctx()
    phi, adj_phi = get_observation_operators(deg_op, path_kernel, r)
    imgs = [read_image(p, ch) for p in path_images]
    groups = {}                                      # same shape -> one device batch
    for i, im in enumerate(imgs):
        groups.setdefault(im.shape, []).append(i)
    per_image = {}
    for shape, idx in groups.items():
        for s in range(0, len(idx), max_batch):
            part = idx[s:s + max_batch]
            xt = np.stack([imgs[i] for i in part])
            xt4 = xt[:, None] if xt.ndim == 3 else xt
            obs, x0 = make_observation_batch(xt4, phi, gaussian_nl, sp_nl, poisson_noise, poisson_alpha, ctx=ctx)
            x, s_sol, c, p, m, t = test_iter_batch(x0, obs, xt4, phi, adj_phi, gamma1, gamma2, alpha_s, alpha_n,
                                                   myLambda, m1, m2, gammaInADMMStep1, gaussian_nl, sp_nl,
                                                   poisson_alpha, path_prox, max_iter, method, ch, r, ctx=ctx)
            for k, i in enumerate(part):
                per_image[i] = (obs[k].reshape(shape), x[k].reshape(shape), s_sol[k].reshape(shape), c[k], p[k],
                                m[k], t / len(part))

    path_saveimg_base = ""
    for index, path_img in enumerate(path_images):
        img_true = imgs[index]
        img_obsrv, img_sol, s_sol, c_evolution, psnr_evolution, ssim_evolution, average_time = per_image[index]
        if poisson_noise:
            img_obsrv = img_obsrv / poisson_alpha                           # main.py:70-71
        filename = os.path.basename(path_img)
        psnr[index] = psnr_evolution[-1]
        ssim[index] = ssim_evolution[-1]
        cpu_time[index] = average_time
        psnr_obsrv, ssim_obsrv = _eval_psnr_ssim(ctx, img_true, img_obsrv)
        results[index] = {"filename": filename, "c_evolution": c_evolution, "PSNR_evolution": psnr_evolution,
                          "SSIM_evolution": ssim_evolution, "GROUND_TRUTH": img_true, "OBSERVATION": img_obsrv,
                          "RESULT": img_sol, "REMOVED_SPARSE": s_sol, "PSNR": psnr_evolution[-1],
                          "SSIM": ssim_evolution[-1], "CPU_time": average_time, "PSNR_observation": psnr_obsrv,
                          "SSIM_observation": ssim_obsrv}
        path_saveimg_base = method + "_" + deg_op + "_" + str(gaussian_nl).ljust(5, "0") + "_(" + filename + ")"
        if add_timestamp:
            path_saveimg_base += "_" + datetime.datetime.now().strftime("%Y%m%d-%H%M%S-%f")
        if save_images:
            save_imgs([img_true, img_obsrv, img_sol],
                      [os.path.join(path_result, k + "_" + path_saveimg_base)
                       for k in ("GROUND_TRUTH", "OBSERVATION", "RESULT")])
        if result_output:
            import matplotlib
            matplotlib.use("Agg")
            import matplotlib.pyplot as plt
            plt.figure()
            plt.title("PSNR")
            plt.plot(np.arange(0, max_iter, 1), psnr_evolution)
            plt.xlabel("iteration")
            plt.ylabel("PSNR")
            plt.savefig(os.path.join(path_result, "PSNR_" + path_saveimg_base + ".png"))
            plt.close()
        if verbose:
            ts = datetime.datetime.now().strftime("%Y/%m/%d %H:%M:%S")
            print(ts + "  (" + str(index + 1) + "/" + str(n_img) + ") PSNR:" + str(psnr[index].round(3)).ljust(6, "0")
                  + "    SSIM:" + str(ssim[index].round(3)).ljust(6, "0") + "   " + filename)

    algorithm, denoiser = get_algorithm_denoiser(method)
    summary = {"Average_PSNR": np.mean(psnr), "PSNR": psnr, "Average_SSIM": np.mean(ssim), "SSIM": ssim,
               "Average_time": np.average(cpu_time), "Cpu_time": cpu_time, "algorithm": algorithm,
               "denoiser": denoiser}
    datas = {"experimental_settings": experimental_settings_all, "method": method_all, "configs": configs_all,
             "results": results, "summary": summary}
    if save_data:
        np.save(os.path.join(path_result, "DATA_" + path_saveimg_base), datas, allow_pickle=True)
    if verbose:
        ts = datetime.datetime.now().strftime("%Y/%m/%d %H:%M:%S")
        print(ts + "  Average_PSNR:" + str(np.mean(psnr).round(3)) + "  Average_SSIM:" + str(np.mean(ssim).round(3))
              + "    Algorithm:" + method + "   Observation:" + deg_op + "   Gaussian noise level:"
              + str(gaussian_nl).ljust(5, "0"))
    return datas


def default_experiments():
    """main.py:107-132: the Experiment-A sweep over noise levels, operators and step sizes."""
    out = []
    for nl in [0.0025, 0.005, 0.01, 0.02, 0.04]:
        for obs in ["blur", "random_sampling"]:
            max_iter = 1200 if obs == "blur" else 3000
            settings = {"gaussian_nl": nl, "sp_nl": 0, "poisson_noise": False, "deg_op": obs, "r": 0.8}
            for method_p in ["A-Proposed", "A-PDS-TV"]:
                for i in range(10):
                    alpha = 0.8 + (i + 1) * 0.02
                    gamma1 = 0.125 if method_p == "A-PDS-TV" else 0.99
                    out.append({"settings": settings, "method": {"method": method_p, "max_iter": max_iter,
                                                                 "gamma1": gamma1, "gamma2": 0.99, "alpha_n": alpha},
                                "configs": {}})
            for method_g in ["A-PnPFBS-DnCNN", "A-RED-DnCNN"]:
                for i in range(10):
                    lam = (i + 1) * 0.2
                    if lam == 2:
                        lam = 1.99
                    out.append({"settings": settings, "method": {"method": method_g, "max_iter": max_iter,
                                                                 "gamma1": 1, "myLambda": lam}, "configs": {}})
    return out


def main(experiment_data_list=None, config=None, **kw):
    """main.py:103-137: run the experiments, one SUMMARY CSV line each."""
    cfg = dict(DEFAULT_CONFIG, **(config or {}))
    os.makedirs(cfg["path_result"], exist_ok=True)
    filepath = os.path.join(cfg["path_result"],
                            "SUMMARY(" + datetime.datetime.now().strftime("%Y%m%d %H%M%S %f") + ").txt")
    touch_textfile(filepath)
    data = None
    for e in (experiment_data_list if experiment_data_list is not None else default_experiments()):
        data = test_all_images(e["settings"], e["method"], e["configs"], config=cfg, **kw)
        write_textfile(filepath, data)
    if data is not None:
        add_footer_textfile(filepath, data)
    return filepath
