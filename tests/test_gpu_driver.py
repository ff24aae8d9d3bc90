"""test_all_images (main.py:16-101) on the device: batched per shape, per-image results equal
to the single-image test_iter run on main.py's observation of that image."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _write_images(d):
    from PIL import Image
    rng = np.random.default_rng(3)
    os.makedirs(d, exist_ok=True)
    for name, (h, w) in (("01.png", (64, 64)), ("02.png", (48, 64)), ("03.png", (64, 64))):
        yy, xx = np.meshgrid(np.linspace(0, 1, h), np.linspace(0, 1, w), indexing="ij")
        img = np.stack([0.5 + 0.3 * np.sin(6 * xx + k) * np.cos(4 * yy) for k in range(3)], -1)
        img += 0.05 * rng.standard_normal(img.shape)
        Image.fromarray(np.uint8(np.clip(img, 0, 1) * 255)).save(os.path.join(d, name))


@pytest.mark.parametrize("settings,method", [
    ({"gaussian_nl": 0.01, "deg_op": "blur"}, {"method": "A-Proposed", "max_iter": 3, "gamma1": 0.99,
                                                "gamma2": 0.99, "alpha_n": 0.95}),
    ({"gaussian_nl": 0.0, "poisson_noise": True, "deg_op": "random_sampling", "r": 0.5},
     {"method": "C-Proposed", "max_iter": 3, "gamma1": 0.00035, "gamma2": 1 / 0.00035}),
])
def test_all_images_matches_single_image_runs(tmp_path, settings, method):
    from pnppds import driver
    from pnppds.iteration import test_iter
    from pnppds.noise import make_observation
    from pnppds.operators import get_observation_operators
    img_dir, res_dir = str(tmp_path / "img"), str(tmp_path / "res")
    _write_images(img_dir)
    cfg = {"root_folder": str(tmp_path), "path_test": img_dir, "path_result": res_dir, "pattern_red": "*.png"}
    datas = driver.test_all_images(settings, method, {"add_timestamp": False}, config=cfg, verbose=False)
    assert len(datas["results"]) == 3
    gn, sp, pois, pa, deg, r = driver.parse_args_exp(settings)
    m = driver.parse_args_method(method)
    phi, adj = get_observation_operators(deg, "blur_1", r)
    for i, res in datas["results"].items():
        xt = driver.read_image(os.path.join(img_dir, res["filename"]), 3)
        obs, x0 = make_observation(xt, deg, "blur_1", r, gn, sp, pois, pa)
        x, s, c, p, ssim, t = test_iter(x0, obs, xt, phi, adj, m[3], m[4], m[6], m[5], m[7], m[8], m[9], m[10],
                                        gn, sp, pa, m[1] + ".pth", m[2], m[0], 3, r)
        np.testing.assert_array_equal(res["PSNR_evolution"], p)
        np.testing.assert_array_equal(res["SSIM_evolution"], ssim)
        np.testing.assert_array_equal(res["RESULT"], x)
        assert res["PSNR"] == p[-1] and np.isfinite(res["SSIM_observation"])
    names = os.listdir(res_dir)
    assert sum(n.startswith("RESULT_") for n in names) == 3
    data_file = [n for n in names if n.startswith("DATA_")]
    assert len(data_file) == 1
    back = np.load(os.path.join(res_dir, data_file[0]), allow_pickle=True).item()   # our own file
    assert back["summary"]["algorithm"] == "PnP-PDS"
    np.testing.assert_allclose(back["summary"]["Average_PSNR"], np.mean([r["PSNR"] for r in datas["results"].values()]))
