"""ORACLE — CPU restatement of the reference PnP-PDS hot path.  TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this module, and only as the checker / the timed CPU baseline.  The product
path (``pnp-pds_amd/``) never imports it and fails loudly without its HIP library.

Pinning: every function here is checked in ``tests/test_oracle_golden.py`` against
golden vectors produced by importing the reference itself in the build container
(``tests/golden/make_golden.py``; fixtures in ``tests/golden/*.npz``).

Semantics follow the reference file:line cited on each function, including its
mixed precision: the denoiser runs in float32 (models/denoiser.py:37) while the
dual variables live in float64 numpy arrays (iteration.py:23-29).
"""
from __future__ import annotations

import time

import numpy as np
import torch
import torch.nn.functional as F

LEAKY_SLOPE = 0.01


# ---------------------------------------------------------------------------
# Observation operators (operators.py:7-79)
# ---------------------------------------------------------------------------
def _kernel_spectrum(h: np.ndarray, shape) -> np.ndarray:
    """FFT of h placed circularly so that tap (a, b) sits at offset (a - m, b - m)."""
    H, W = shape
    kh, kw = h.shape
    hp = np.zeros((H, W), np.float64)
    for a in range(kh):
        for b in range(kw):
            if h[a, b] != 0.0:
                hp[(a - kh // 2) % H, (b - kw // 2) % W] += h[a, b]
    return np.fft.fft2(hp)


def blur(x: np.ndarray, h: np.ndarray) -> np.ndarray:
    """Φx — operators.py:7-22.  The reference's wrap-pad + FFT + crop equals the centred
    circular convolution  y[i,j] = Σ_ab h[a,b] x[(i-a+m) mod H, (j-b+m) mod W]."""
    A = _kernel_spectrum(h, x.shape[-2:])
    return np.real(np.fft.ifft2(np.fft.fft2(np.asarray(x, np.float64)) * A))


def adj_blur(x: np.ndarray, h: np.ndarray) -> np.ndarray:
    """Φᵀx — operators.py:24-38: circular correlation  y[i,j] = Σ_ab h[a,b] x[(i+a-m), (j+b-m)]."""
    A = _kernel_spectrum(h, x.shape[-2:])
    return np.real(np.fft.ifft2(np.fft.fft2(np.asarray(x, np.float64)) * np.conj(A)))


def sampling_mask(H: int, W: int, r: float) -> np.ndarray:
    """Keep-mask of operators.py:40-58: round(H·W·(1-r)) pixels dropped, chosen by
    RandomState(1234).permutation(H·W), shared by all channels.  Returns uint8 [H, W]."""
    cnt = round(H * W * (1 - r))
    q = np.random.RandomState(seed=1234).permutation(H * W)[:cnt]
    m = np.ones(H * W, np.uint8)
    m[q] = 0
    return m.reshape(H, W)


def random_sampling(x: np.ndarray, r: float) -> np.ndarray:
    """operators.py:40-58 (self-adjoint); returns float64 like the reference."""
    m = sampling_mask(x.shape[-2], x.shape[-1], r)
    return np.where(m.astype(bool), np.asarray(x, np.float64), 0.0)   # t[q] = 0: NaN-safe like the shipped code


def observation_operators(kind: str, h: np.ndarray | None = None, r: float = 0.8):
    """(phi, adj_phi) — operators.py:60-79."""
    if kind == "blur":
        return (lambda x: blur(x, h)), (lambda x: adj_blur(x, h))
    if kind == "random_sampling":
        f = lambda x: random_sampling(x, r)  # noqa: E731
        return f, f
    if kind == "Id":
        return (lambda x: x), (lambda x: x)
    raise ValueError(kind)


# ---------------------------------------------------------------------------
# Proximal operators (operators.py:94-115) and metrics (utils/utils_eval.py:4-7)
# ---------------------------------------------------------------------------
def proj_l1_ball(x, alpha_s, sp_nl, r=1):
    """operators.py:94-100: Euclidean projection onto {‖s‖₁ ≤ η}, η = α_s·N·sp_nl·r/2,
    with θ = max(0, max_k (S_k − η)/k) over |x| sorted descending."""
    eta = alpha_s * x.size * sp_nl * r * 0.5
    a = np.abs(np.ravel(x))
    srt = np.sort(a)[::-1]
    theta = np.max((np.cumsum(srt) - eta) / np.arange(1, a.size + 1))
    theta = max(theta, 0.0)
    return (np.fmax(a - theta, 0) * np.sign(np.ravel(x))).reshape(x.shape)


def proj_l2_ball(x, alpha_n, gaussian_nl, sp_nl, x_0, r=1):
    """operators.py:102-108: projection onto the ball B(x_0, ε), ε = sqrt(N(1-sp_nl))·r·α_n·σ."""
    eps = np.sqrt(x.size * (1 - sp_nl)) * r * alpha_n * gaussian_nl
    d = x - x_0
    nrm = np.linalg.norm(d)
    if nrm > eps:
        return x_0 + eps * d / nrm
    return np.copy(x)


def prox_gkl(x, gamma, alpha, x_0):
    """operators.py:114-115 (generalised-KL prox), elementwise."""
    t = x - gamma * alpha
    return 0.5 * (t + np.sqrt(np.square(t) + 4 * gamma * x_0))


def psnr(x_true, x):
    """utils/utils_eval.py:4-7 (data_range 1, float64 MSE)."""
    mse = np.mean((np.asarray(x_true, np.float64) - np.asarray(x, np.float64)) ** 2)
    return 10 * np.log10(1.0 / mse)


def _ssim_single(im1, im2, data_range, win_size=7):
    """skimage.metrics.structural_similarity (scikit-image 0.22.0, pinned in the reference's
    requirements.txt), channel_axis=None path, default arguments: uniform 7-wide window
    (scipy.ndimage.uniform_filter, axis by axis), K1 = 0.01, K2 = 0.03, sample covariance,
    float32 arithmetic for float32 inputs, mean over the map cropped by (win-1)/2."""
    from scipy.ndimage import uniform_filter
    ft = np.float32
    im1 = im1.astype(ft, copy=False)
    im2 = im2.astype(ft, copy=False)
    NP = win_size ** im1.ndim
    cov_norm = NP / (NP - 1)
    ux = uniform_filter(im1, size=win_size)
    uy = uniform_filter(im2, size=win_size)
    uxx = uniform_filter(im1 * im1, size=win_size)
    uyy = uniform_filter(im2 * im2, size=win_size)
    uxy = uniform_filter(im1 * im2, size=win_size)
    vx = cov_norm * (uxx - ux * ux)
    vy = cov_norm * (uyy - uy * uy)
    vxy = cov_norm * (uxy - ux * uy)
    R = data_range
    C1 = (0.01 * R) ** 2
    C2 = (0.03 * R) ** 2
    A1, A2, B1, B2 = (2 * ux * uy + C1, 2 * vxy + C2, ux ** 2 + uy ** 2 + C1, vx + vy + C2)
    S = (A1 * A2) / (B1 * B2)
    pad = (win_size - 1) // 2
    crop = tuple(slice(pad, n - pad) for n in S.shape)
    return S[crop].mean(dtype=np.float64)


def ssim(x_true, x):
    """utils/utils_eval.py:9-12: structural_similarity(x_true, x, data_range = x.max() -
    x.min(), channel_axis=0).  channel_axis=0 makes skimage loop over axis 0 and average:
    an RGB (C,H,W) image gives the mean of C 2-D SSIMs; a grayscale (H,W) image gives the
    mean of H 1-D SSIMs over its rows (the reference's quirk).
    PARITY UNPINNED: scikit-image is absent here, so this restatement of its published
    algorithm is checked against no reference output."""
    x_true = np.asarray(x_true, np.float32)
    x = np.asarray(x, np.float32)
    data_range = x.max() - x.min()
    vals = np.array([_ssim_single(x_true[i], x[i], data_range) for i in range(x.shape[0])], np.float32)
    return float(vals.mean())


# ---------------------------------------------------------------------------
# Observation pipeline (main.py:49-64, utils/utils_noise.py) — numpy legacy RandomState,
# the generator the reference itself calls (numpy's legacy stream is frozen across versions).
# ---------------------------------------------------------------------------
def add_gaussian_noise(img, noise_level, op):
    """utils_noise.py:35-38."""
    rs = np.random.RandomState(1234)
    return img + op(noise_level * rs.randn(*img.shape))


def apply_poisson_noise(img, alpha):
    """utils_noise.py:40-43."""
    rs = np.random.RandomState(1234)
    return rs.poisson(img * alpha)


def add_salt_and_pepper_noise(img, noise_level, op):
    """utils_noise.py:3-33, with the O(n^2) list membership replaced by a set.  The loop's
    ``i=i-1`` has no effect in a Python for-loop: exactly 2*noise_cnt pairs are drawn, the
    accepted ones (target pixel == 1, first occurrence) become 0 (first noise_cnt) or 1.
    Both coordinates are drawn in [0, img.shape[-2]) and keyed x*shape[-2]+y (as shipped)."""
    H, W = img.shape[-2], img.shape[-1]
    noise_cnt = int(H * W * noise_level / 2)
    target = op(np.ones([H, W]))
    rs = np.random.RandomState(1234)
    seen, xs, ys = set(), [], []
    for _ in range(noise_cnt * 2):
        x = rs.randint(0, H)
        y = rs.randint(0, H)
        key = x * H + y
        if target[x][y] == 1 and key not in seen:
            seen.add(key)
            xs.append(x)
            ys.append(y)
    xs, ys = np.array(xs, dtype=np.int64), np.array(ys, dtype=np.int64)
    out = np.copy(img)
    planes = [out] if out.ndim == 2 else [out[c] for c in range(3)]
    for pl in planes:
        pl[(xs[:noise_cnt], ys[:noise_cnt])] = 0
        pl[(xs[noise_cnt:], ys[noise_cnt:])] = 1
    return out


def make_observation(x_true, deg_op, h, r, gaussian_nl, sp_nl, poisson_noise, poisson_alpha):
    """main.py:49-64: returns (img_obsrv, x_0) with the reference's dtypes."""
    phi, _ = observation_operators(deg_op, h, r)
    ident = (lambda v: v)
    noise_op = ident if deg_op in ("blur", "Id") else phi
    obs = phi(x_true)
    obs = add_gaussian_noise(obs, gaussian_nl, noise_op)
    if poisson_noise:
        obs = apply_poisson_noise(obs, poisson_alpha)
    obs = add_salt_and_pepper_noise(obs, sp_nl, noise_op)
    x0 = np.copy(obs)
    if poisson_noise:
        x0 = x0 / poisson_alpha
    return obs, x0


# ---------------------------------------------------------------------------
# Denoiser (models/denoiser.py:34-46, models/basic_models.py:25-38,
#           KAIR variant models/network_dncnn.py:42-77)
# ---------------------------------------------------------------------------
def fp16_filter_round(w):
    """The fp16 values the device stores for conv weights w [c_out, c_in, 3, 3] (capi.hip
    fp16_filter_round; device numerics, not a reference function): round to nearest, then per
    3x3 filter move taps to their other fp16 neighbour, cheapest added error first (lowest tap
    index on ties), while a move shrinks |sum of the filter's rounding errors|.  Returns float32
    arrays of fp16-representable values."""
    w = np.ascontiguousarray(w, np.float32)
    f = w.reshape(-1, 9).astype(np.float64)
    h = w.reshape(-1, 9).astype(np.float16)
    r = h.astype(np.float64)
    up = np.nextafter(h, np.float16(np.inf)).astype(np.float64)
    dn = np.nextafter(h, np.float16(-np.inf)).astype(np.float64)
    alt = np.where(r == f, r, np.where(r < f, up, dn))
    cost = np.abs(alt - f) - np.abs(r - f)
    S = (r - f).sum(1)                              # exact: a few dozen bits span
    used = np.zeros(r.shape, bool)
    rows = np.arange(r.shape[0])
    for _ in range(9):
        d = alt - r
        cand = ~used & (np.abs(S[:, None] + d) < np.abs(S)[:, None])
        any_c = cand.any(1)
        if not any_c.any():
            break
        j = np.argmin(np.where(cand, cost, np.inf), 1)
        sel = rows[any_c]
        js = j[any_c]
        S[sel] += d[sel, js]
        r[sel, js] = alt[sel, js]
        used[sel, js] = True
    return r.astype(np.float32).reshape(w.shape)


class OracleDenoiser:
    """Forward of the conv stack on torch-CPU in float32.

    ``emulate_fp16=True`` rounds every conv's input activations to fp16 and takes the weights'
    fp16 values from ``fp16_filter_round`` (fp32 accumulation, fp16 storage of hidden
    activations) — the device numerics of PNP_PREC_FP16.  ``emulate_fp16="w2"``: activations
    rounded to fp16, weights as the sum of that fp16 high half and the fp16 rounding of the
    remainder (PNP_PREC_FP16W2).  ``emulate_fp16="a2"``: activations kept (the device's hi + lo
    pairs carry ~21 bits), the 64 -> 64 layers' weights at their fp16 values, head and tail
    exact (PNP_PREC_FP16A2).
    """

    def __init__(self, weights, emulate_fp16=False):
        self.w = weights
        self.emulate_fp16 = emulate_fp16 in (True, "w2")      # fp16 activations
        self.tw = [torch.from_numpy(np.ascontiguousarray(a, np.float32)) for a in weights.weights]
        self.tb = [torch.from_numpy(np.ascontiguousarray(b, np.float32)) for b in weights.biases]
        if emulate_fp16:                     # the device's fp16 weights (fp16_filter_round)
            hi = [torch.from_numpy(fp16_filter_round(t.numpy())) for t in self.tw]
            if emulate_fp16 == "w2":          # + the fp16 rounding of the remainder
                self.tw = [a + (t - a).half().float() for a, t in zip(hi, self.tw)]
            elif emulate_fp16 == "a2":        # fp16 body weights only
                self.tw = [hi[i] if 0 < i < len(hi) - 1 else t for i, t in enumerate(self.tw)]
            else:
                self.tw = hi

    @torch.no_grad()
    def forward_batch(self, x: np.ndarray) -> np.ndarray:
        """x: [B, C, H, W] -> [B, C, H, W] float32."""
        xin = torch.from_numpy(np.ascontiguousarray(x, np.float32))
        if self.w.clamp_io:
            xin = xin.clamp(0, 1)
        h = xin
        n = len(self.tw)
        for i in range(n):
            if self.emulate_fp16:
                h = h.half().float()
            h = F.conv2d(h, self.tw[i], self.tb[i], padding=1)
            if i < n - 1:
                h = F.leaky_relu(h, LEAKY_SLOPE) if self.w.act == 0 else F.relu(h)
        out = h + xin if self.w.residual > 0 else xin - h
        if self.w.clamp_io:
            out = out.clamp(0, 1)
        return out.numpy()

    def denoise(self, x: np.ndarray) -> np.ndarray:
        """Reference call shape: (C,H,W) for RGB, (H,W) for gray (denoiser.py:35-36)."""
        if x.ndim == 2:
            return self.forward_batch(x[None, None])[0, 0]
        return self.forward_batch(x[None])[0]


# ---------------------------------------------------------------------------
# test_iter (iteration.py:10-196), methods A/B/C-Proposed and comparisonB-2
# ---------------------------------------------------------------------------
METHOD_ALIASES = {"ours-A": "A-Proposed", "ours-B": "B-Proposed", "ours-C": "C-Proposed"}


# ---------------------------------------------------------------------------
# TV operators (operators.py:110-137) — restated with the shipped boundary handling
# ---------------------------------------------------------------------------
def D(x):
    """operators.py:120-126: forward differences along rows then columns, zero last row /
    column; (C,H,W) -> (2C,H,W)."""
    xv = np.zeros(x.shape)
    xh = np.zeros(x.shape)
    xv[:, :-1, :] = x[:, 1:, :] - x[:, :-1, :]
    xh[:, :, :-1] = x[:, :, 1:] - x[:, :, :-1]
    return np.concatenate([xv, xh], 0)


def D_T(y):
    """operators.py:128-137 as shipped: first row -y[0], inner rows y[i-1] - y[i], last row
    +y[H-1] (not y[H-2]); likewise for columns."""
    C = y.shape[0] // 2
    yv, yh = y[:C], y[C:]
    ov = np.empty(yv.shape)
    ov[:, 0] = -yv[:, 0]
    ov[:, 1:-1] = -yv[:, 1:-1] + yv[:, :-2]
    ov[:, -1] = yv[:, -1]
    oh = np.empty(yh.shape)
    oh[:, :, 0] = -yh[:, :, 0]
    oh[:, :, 1:-1] = -yh[:, :, 1:-1] + yh[:, :, :-2]
    oh[:, :, -1] = yh[:, :, -1]
    return ov + oh


def prox_l12(x, gamma):
    """operators.py:110-112: per-pixel group soft threshold over axis 0."""
    with np.errstate(divide="ignore"):
        val = gamma / np.sqrt(np.sum(x * x, 0))
    return np.fmax(1 - val, 0) * x


def _admm_poisson_x(u, v, y, phi, adj_phi, alpha, lam, m, gamma):
    """algorithm/admm.py:4-16 (step1ofADMMforPoisson)."""
    x = np.ones(u.shape)
    for _ in range(m):
        with np.errstate(divide="ignore", invalid="ignore"):
            ratio = y / (alpha * phi(x))
        grad = -adj_phi(ratio) / alpha + adj_phi(np.ones(x.shape)) / alpha + lam * (x - v + u)
        x = x - gamma * grad
    return x


def test_iter(x_0, x_obsrv, x_true, phi, adj_phi, gamma1, gamma2, alpha_s, alpha_n, myLambda,
              m1, m2, gammaInADMMStep1, gaussian_nl, sp_nl, poisson_alpha, denoiser, max_iter,
              method="A-Proposed", ch=3, r=1, ssim_fn=None):
    """Restatement of iteration.test_iter for the hot-path methods.  ``denoiser`` is an
    OracleDenoiser (the reference builds one from ``path_prox``, iteration.py:40-41)."""
    method = METHOD_ALIASES.get(method, method)
    x_n = x_0
    y_n = np.zeros(x_0.shape)
    y1_n = np.zeros((2 * x_0.shape[0],) + x_0.shape[1:]) if x_0.ndim == 3 else None
    y2_n = np.zeros(x_0.shape)
    s_n = np.zeros(x_0.shape)
    z_n = np.zeros(x_0.shape)
    d_n = np.zeros(x_0.shape)
    c = np.zeros(max_iter)
    psnr_data = np.zeros(max_iter)
    ssim_data = np.zeros(max_iter)
    t0 = time.perf_counter()
    for i in range(max_iter):
        x_prev = x_n
        s_prev = s_n
        if method == "A-Proposed":                                        # iteration.py:48-52
            x_n = denoiser.denoise(x_n - gamma1 * adj_phi(y_n))
            y_n = y_n + gamma2 * phi(2 * x_n - x_prev)
            y_n = y_n - gamma2 * proj_l2_ball(y_n / gamma2, alpha_n, gaussian_nl, sp_nl, x_obsrv)
        elif method == "B-Proposed":                                      # iteration.py:53-58
            x_n = denoiser.denoise(x_n - gamma1 * adj_phi(y_n))
            s_n = proj_l1_ball(s_n - gamma1 * y_n, alpha_s, sp_nl, r)
            y_n = y_n + gamma2 * (phi(2 * x_n - x_prev) + 2 * s_n - s_prev)
            y_n = y_n - gamma2 * proj_l2_ball(y_n / gamma2, alpha_n, gaussian_nl, sp_nl, x_obsrv, r)
        elif method == "C-Proposed":                                      # iteration.py:59-63
            x_n = denoiser.denoise(x_n - gamma1 * adj_phi(y_n))
            y_n = y_n + gamma2 * phi(2 * x_n - x_prev)
            y_n = y_n - gamma2 * prox_gkl(y_n / gamma2, myLambda / gamma2, poisson_alpha, x_obsrv)
        elif method == "comparisonB-2":                                   # iteration.py:127-132
            x_n = np.ones(s_n.shape)                                      # admm.py:30-36
            for _ in range(m1):
                x_n = x_n - 1 / gamma1 * adj_phi(phi(x_n) + s_n - z_n + y_n)
                x_n = denoiser.denoise(x_n)
            s_n = np.ones(x_n.shape)                                      # admm.py:38-44
            for _ in range(m2):
                s_n = s_n - 1 / gamma1 * (phi(x_n) + s_n - z_n + y_n)
                s_n = proj_l1_ball(s_n, alpha_s, sp_nl)
            z_n = proj_l2_ball(phi(x_n) + s_n + y_n, alpha_n, gaussian_nl, sp_nl, x_obsrv)
            y_n = y_n + phi(x_n) + s_n - z_n
        elif method == "A-PnPFBS-DnCNN":                                  # iteration.py:71-73
            x_n = denoiser.denoise(x_n - gamma1 * myLambda * 0.5 * (2 * adj_phi(phi(x_n) - x_obsrv)))
        elif method == "A-PDS-TV":                                        # iteration.py:86-91
            x_n = x_n - gamma1 * (D_T(y1_n) + adj_phi(y2_n))
            y1_n = y1_n + gamma2 * D(2 * x_n - x_prev)
            y1_n = y1_n - gamma2 * prox_l12(y1_n / gamma2, 1 / gamma2)
            y2_n = y2_n + gamma2 * (phi(2 * x_n - x_prev))
            y2_n = y2_n - gamma2 * proj_l2_ball(y2_n / gamma2, alpha_n, gaussian_nl, sp_nl, x_obsrv)
        elif method == "A-FBS-TV":                                        # iteration.py:92-96
            x_n = x_n - gamma1 * (adj_phi(phi(x_n) - x_obsrv) + D_T(y1_n))
            y1_n = y1_n + gamma2 * D(2 * x_n - x_prev)
            y1_n = y1_n - gamma2 * prox_l12(y1_n / gamma2, 1 / gamma2)
        elif method == "A-RED-DnCNN":                                     # iteration.py:97-103
            x_n = denoiser.denoise(x_n)
            mu = 2 / (1 / gamma1 ** 2 + myLambda)
            x_n = x_prev - mu * ((1 / gamma1 ** 2) * adj_phi(phi(x_prev) - x_obsrv) + myLambda * (x_prev - x_n))
        elif method in ("A-PnPPDS-unstable-DnCNN", "C-PnP-unstable-DnCNN"):   # iteration.py:104-110,174-180
            x_n = denoiser.denoise(x_n - gamma1 * adj_phi(y_n))          # denoiser = the KAIR DnCNN here
            y_n = y_n + gamma2 * phi(2 * x_n - x_prev)
            if method.startswith("A"):
                y_n = y_n - gamma2 * proj_l2_ball(y_n / gamma2, alpha_n, gaussian_nl, sp_nl, x_obsrv)
            else:
                y_n = y_n - gamma2 * prox_gkl(y_n / gamma2, myLambda / gamma2, poisson_alpha, x_obsrv)
        elif method == "comparisonB-3":                                   # iteration.py:139-145
            x_n = x_n - gamma1 * (D_T(y1_n) + adj_phi(y2_n))
            s_n = proj_l1_ball(s_n - gamma1 * y2_n, alpha_s, sp_nl)
            y1_n = y1_n + gamma2 * D(2 * x_n - x_prev)
            y1_n = y1_n - gamma2 * prox_l12(y1_n / gamma2, 1 / gamma2)
            y2_n = y2_n + gamma2 * (phi(2 * x_n - x_prev) + 2 * s_n - s_prev)
            y2_n = y2_n - gamma2 * proj_l2_ball(y2_n / gamma2, alpha_n, gaussian_nl, sp_nl, x_obsrv)
        elif method == "comparisonB-4":                                   # iteration.py:146-151
            x_n = x_prev - gamma1 * (myLambda * adj_phi(phi(x_prev) + s_n - x_obsrv) + (x_prev - denoiser.denoise(x_n)))
            s_n = proj_l1_ball(s_n - gamma1 * (phi(x_n) + s_n - x_obsrv), alpha_s, sp_nl)
        elif method == "comparisonB-5":                                   # iteration.py:152-155
            x_n = denoiser.denoise(x_n - gamma1 * (2 * adj_phi(phi(x_n) + s_n - x_obsrv)))
            s_n = proj_l1_ball(s_n - gamma1 * (phi(x_n) + s_n - x_obsrv), alpha_s, sp_nl)
        elif method in ("C-PnPADMM-DnCNN", "C-RED-DnCNN"):                # iteration.py:163-173
            x_n = _admm_poisson_x(d_n, z_n, x_obsrv, phi, adj_phi, poisson_alpha, myLambda, m1, gammaInADMMStep1)
            if method == "C-PnPADMM-DnCNN":
                z_n = denoiser.denoise(x_n + d_n)
            else:                                                         # admm.py:18-27 (beta=myLambda, lam=gamma1)
                z_str = x_n + d_n
                for _ in range(m2):
                    z_n = denoiser.denoise(z_n)
                    z_n = 1 / (myLambda + gamma1) * (gamma1 * z_n + myLambda * z_str)
            d_n = d_n + x_n - z_n
        else:
            raise ValueError(f"Unknown method: {method}")
        c[i] = np.linalg.norm((x_n - x_prev).flatten(), 2) / np.linalg.norm(x_prev.flatten(), 2)
        psnr_data[i] = psnr(x_true, x_n)
        if ssim_fn is not None:
            ssim_data[i] = ssim_fn(x_true, x_n)
    avg = (time.perf_counter() - t0) / max(max_iter, 1)
    return x_n, s_n + 0.5, c, psnr_data, ssim_data, avg
