"""Which fp16 rounding drives the ours-C drift?  Oracle test_iter with fp16 rounding emulated in
parts of the denoiser (none / weights / activations / input only / both), |dPSNR| against the
reference trajectory tests/golden/long_C_rs_3000.npz.  CPU only (profiling aid).

    python tools/precision_drift_emu.py {none,w,a,in,both,w2a} 1000
    (w2a: fp16 activations with weights split into fp16 hi + lo pairs)
"""
import os, sys, numpy as np, torch
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, 'pnp-pds_amd'), os.path.join(REPO, 'tests')]
torch.set_num_threads(2)
import torch.nn.functional as F
from oracle import pnp_oracle as O
from pnppds.weights import resolve_weights
from pnppds.operators import load_blur_kernel
mode = sys.argv[1]; iters = int(sys.argv[2])
class Emu(O.OracleDenoiser):
    def __init__(self, w, rw, ra, first_only=False):
        super().__init__(w)
        self.ra, self.first_only = ra, first_only
        if rw == 1: self.tw = [t.half().float() for t in self.tw]
        if rw == 2:   # fp16 hi + fp16 lo split (lo = fp16(w - hi), subnormals kept): fp16x2 weights
            self.tw = [t.half().float() + (t - t.half().float()).half().float() for t in self.tw]
    @torch.no_grad()
    def forward_batch(self, x):
        xin = torch.from_numpy(np.ascontiguousarray(x, np.float32)).clamp(0, 1)
        h = xin; n = len(self.tw)
        for i in range(n):
            if self.ra and not (self.first_only and i > 0): h = h.half().float()
            h = F.conv2d(h, self.tw[i], self.tb[i], padding=1)
            if i < n - 1: h = F.leaky_relu(h, 0.01)
        return (h + xin).clamp(0, 1).numpy()
rw, ra, fo = {'none': (0,0,0), 'w': (1,0,0), 'a': (0,1,0), 'both': (1,1,0), 'in': (0,1,1),
              'w2a': (2,1,0)}[mode]
z = np.load(os.path.join(REPO, 'tests/golden/long_C_rs_3000.npz'))
den = Emu(resolve_weights('DnCNN_nobn_nch_3_nlev_0.01', 3), rw, ra, fo)
p = z['params']; g1, g2, as_, an, lam, m1, m2, gad, sig, sp, pa, _, ch, r = p
phi, adj = O.observation_operators('random_sampling', None, r)
res = O.test_iter(z['x_0'].astype(np.float64), z['x_obs'].astype(np.float64), z['x_true'], phi, adj, g1, g2, as_, an, lam, int(m1), int(m2), gad, sig, sp, pa, den, iters, 'C-Proposed', 3, r)
d = np.abs(res[3] - z['psnr'][:iters])
print(mode, 'max', d.max(), 'at', [round(float(d[i]),5) for i in (99, 299, iters//2, iters-1)], flush=True)
