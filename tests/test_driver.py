"""Driver / results format vs the reference's own utils_textfile.py,
utils_parse_args.py and utils_method_master.py outputs (tests/golden/driver.json)."""
import json
import os

import numpy as np
import pytest

from pnppds import driver

GOLD = os.path.join(os.path.dirname(__file__), "golden", "driver.json")


@pytest.fixture(scope="module")
def gold():
    with open(GOLD) as f:
        return json.load(f)


def test_csv_text_matches_reference(gold):
    datas = dict(gold["datas"])
    datas["results"] = {i: r for i, r in enumerate(gold["results"])}
    assert driver.get_csv_header() == gold["header"]
    assert driver.get_csv_data(datas) == gold["data"]
    assert driver.get_csv_footer(datas) == gold["footer"]


def test_argument_defaults_match_reference(gold):
    assert list(driver.parse_args_exp({})) == gold["defaults"]["exp"]
    assert list(driver.parse_args_method({})) == gold["defaults"]["method"]
    assert list(driver.parse_args_configs({})) == gold["defaults"]["configs"]
    for m, want in gold["methods"].items():
        assert list(driver.get_algorithm_denoiser(m)) == want


def test_textfile_roundtrip(tmp_path, gold):
    datas = dict(gold["datas"])
    datas["results"] = {i: r for i, r in enumerate(gold["results"])}
    f = tmp_path / "SUMMARY.txt"
    driver.touch_textfile(f)
    driver.write_textfile(f, datas)
    driver.add_footer_textfile(f, datas)
    assert f.read_text() == gold["header"] + gold["data"] + "\n" + gold["footer"] + "\n"


def test_image_io_bgr_order(tmp_path):
    from PIL import Image
    rgb = np.zeros((4, 5, 3), np.uint8)
    rgb[..., 0], rgb[..., 1], rgb[..., 2] = 255, 128, 0          # R, G, B
    Image.fromarray(rgb).save(tmp_path / "a.png")
    x = driver.read_image(str(tmp_path / "a.png"), 3)
    assert x.shape == (3, 4, 5) and x.dtype == np.float32
    np.testing.assert_array_equal(x[0], 0.0)                      # cv2 order: B, G, R
    np.testing.assert_array_equal(x[2], 1.0)
    g = driver.read_image(str(tmp_path / "a.png"), 1)
    assert g.shape == (4, 5)
    np.testing.assert_allclose(g, 0.299 + 0.587 * 128 / 255, rtol=1e-6)
    driver.save_img(x, str(tmp_path / "b"))                       # utils_image.save_img round trip
    np.testing.assert_array_equal(np.asarray(Image.open(tmp_path / "b.png")), rgb)


def test_default_sweep_is_main_py():
    e = driver.default_experiments()
    assert len(e) == 5 * 2 * 4 * 10
    assert e[0]["method"] == {"method": "A-Proposed", "max_iter": 1200, "gamma1": 0.99, "gamma2": 0.99,
                              "alpha_n": 0.8 + 0.02}
    assert e[10]["method"]["gamma1"] == 0.125 and e[10]["method"]["method"] == "A-PDS-TV"
    assert e[39]["method"]["myLambda"] == 1.99
