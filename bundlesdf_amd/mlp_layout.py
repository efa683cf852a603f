"""MFMA operand layout of the fused tiny MLP (NeRFSmall: nerf_helpers.py:243-321,
built at nerf_runner.py:221 with num_layers=2, hidden 64, geo 15, colour 3
layers, input 32 = L*C, views 9 = SH degree 3).

The fused field kernel (csrc/field_step.hip) keeps activations transposed —
features on MFMA rows (accumulator registers), the wave's 32 samples on MFMA
columns (lanes) — and runs v_mfma_f32_32x32x16_f16 (amp) or
v_mfma_f32_32x32x2_f32 (fp32) tiles. A layer whose input is the previous
layer's accumulator uses it as the B operand in place (no LDS), which permutes
the K order inside each 16-wide step; the weights (A operand) are pre-packed
here with the same permutation:

  32x32x16 lane l: m = l & 31, h = l >> 5, element j in 0..7
  acc row of register q, half h:   (q & 3) + 8 (q >> 2) + 4 h
  natural K step s:                k = 16 s + 8 h + j        (only the dlogit operand)
  accumulator K step (t, s):       k = 32 t + 16 s + 8 (j >> 2) + 4 h + (j & 3)

Layer 1 also uses the accumulator order: lane (n, h) encodes exactly the
levels whose features are its accumulator rows, so the encoder output is the
B operand in place and the layer-1 backward accumulator is the scatter input.

The colour MLP input is re-ordered to reuse the sigma head's accumulator:
Cin row 0 (= sdf) gets weight 0, rows 1..15 = geo features, rows 16..24 = the
9 SH coefficients, rows 25..25+ff-1 = the ray's frame features (cfg
frame_features = ff <= 3; the reference's colour input is [frame features, SH,
geo], nerf_runner.py:221,1277 / nerf_helpers.py:310-316), the rest 0.
"""
import numpy as np

IN, HID, GEO, VIEWS = 32, 64, 15, 9        # IN = L * C (<= 32; W1 K-columns beyond it are zero)
MLP_KEYS = ["sigma_net.0.weight", "sigma_net.0.bias", "sigma_net.2.weight", "sigma_net.2.bias",
            "color_net.0.weight", "color_net.0.bias", "color_net.2.weight", "color_net.2.bias",
            "color_net.4.weight", "color_net.4.bias"]


def shapes(n_in=IN, ff=0):
    return {"sigma_net.0.weight": (HID, n_in), "sigma_net.0.bias": (HID,), "sigma_net.2.weight": (1 + GEO, HID),
            "sigma_net.2.bias": (1 + GEO,), "color_net.0.weight": (HID, ff + VIEWS + GEO), "color_net.0.bias": (HID,),
            "color_net.2.weight": (HID, HID), "color_net.2.bias": (HID,), "color_net.4.weight": (3, HID),
            "color_net.4.bias": (3,)}


def offsets(n_in=IN, ff=0):
    off, o, sh = {}, 0, shapes(n_in, ff)
    for k in MLP_KEYS:
        off[k] = o
        o += int(np.prod(sh[k]))
    return off, o


SHAPES = shapes()
OFF, N_MLP = offsets()          # N_MLP = 9107 at n_in = 32


def _acc_k(t, s, j, h):
    return 32 * t + 16 * s + 8 * (j >> 2) + 4 * h + (j & 3)


def _nat_k(s, j, h):
    return 16 * s + 8 * h + j


def cin_to_w3_col(k, ff=0):
    """Cin row k -> column of color_net.0.weight (reference input = [frame features(ff), SH(9), geo(15)])."""
    if 1 <= k <= 15:
        return ff + VIEWS + (k - 1)
    if 16 <= k <= 24:
        return ff + k - 16
    if 25 <= k < 25 + ff:
        return k - 25
    return -1


# Fragment list: (name, n_mtiles, ksteps, element index fn(mt, ks, m, h, j) -> flat param index or -1)
def _frag_specs(n_in=IN, ff=0):
    sh, off = shapes(n_in, ff), offsets(n_in, ff)[0]

    def w(key, r, c):
        R, C = sh[key]
        if r < 0 or c < 0 or r >= R or c >= C:
            return -1
        return off[key] + r * C + c

    S = []
    # forward
    S.append(("L1", 2, [(0, s) for s in range(2)],
              lambda mt, t, s, m, h, j: w("sigma_net.0.weight", 32 * mt + m, _acc_k(0, s, j, h))))
    S.append(("L2", 1, [(t, s) for t in range(2) for s in range(2)],
              lambda mt, t, s, m, h, j: w("sigma_net.2.weight", 32 * mt + m, _acc_k(t, s, j, h))))
    S.append(("L3", 2, [(0, s) for s in range(2)],
              lambda mt, t, s, m, h, j: w("color_net.0.weight", 32 * mt + m, cin_to_w3_col(_acc_k(t, s, j, h), ff))))
    S.append(("L4", 2, [(t, s) for t in range(2) for s in range(2)],
              lambda mt, t, s, m, h, j: w("color_net.2.weight", 32 * mt + m, _acc_k(t, s, j, h))))
    S.append(("L5", 1, [(t, s) for t in range(2) for s in range(2)],
              lambda mt, t, s, m, h, j: w("color_net.4.weight", 32 * mt + m, _acc_k(t, s, j, h))))
    # backward data (A = W^T)
    S.append(("B5", 2, [(0, 0)],
              lambda mt, t, s, m, h, j: w("color_net.4.weight", _nat_k(0, j, h), 32 * mt + m)))
    S.append(("B4", 2, [(t, s) for t in range(2) for s in range(2)],
              lambda mt, t, s, m, h, j: w("color_net.2.weight", _acc_k(t, s, j, h), 32 * mt + m)))
    S.append(("B3", 1, [(t, s) for t in range(2) for s in range(2)],
              lambda mt, t, s, m, h, j: w("color_net.0.weight", _acc_k(t, s, j, h), cin_to_w3_col(32 * mt + m, ff))))
    S.append(("B2", 2, [(0, s) for s in range(2)],
              lambda mt, t, s, m, h, j: w("sigma_net.2.weight", _acc_k(t, s, j, h), 32 * mt + m)))
    S.append(("B1", 1, [(t, s) for t in range(2) for s in range(2)],
              lambda mt, t, s, m, h, j: w("sigma_net.0.weight", _acc_k(t, s, j, h), 32 * mt + m)))
    return S


def frag_table(n_in=IN, ff=0):
    """int32 [n_frags, 64, 8] flat-param indices (-1 = zero) and {name: first frag id}.
    Fragment id of (layer, mt, kstep) = base + mt * n_ksteps + kstep."""
    specs = _frag_specs(n_in, ff)
    tabs, base, cur = [], {}, 0
    for name, nmt, ks, fn in specs:
        base[name] = cur
        for mt in range(nmt):
            for (t, s) in ks:
                f = np.full((64, 8), -1, np.int32)
                for lane in range(64):
                    m, h = lane & 31, lane >> 5
                    for j in range(8):
                        f[lane, j] = fn(mt, t, s, m, h, j)
                tabs.append(f)
                cur += 1
    return np.stack(tabs), base


BIAS_LAYERS = ["sigma_net.0.bias", "sigma_net.2.bias", "color_net.0.bias", "color_net.2.bias", "color_net.4.bias"]


def bias_table(n_in=IN, ff=0):
    """int32 [5, 64]: bias image rows (zero padded)."""
    sh, off = shapes(n_in, ff), offsets(n_in, ff)[0]
    t = np.full((5, 64), -1, np.int32)
    for i, k in enumerate(BIAS_LAYERS):
        n = sh[k][0]
        t[i, :n] = off[k] + np.arange(n)
    return t


def pack_table(n_in=IN, ff=0):
    """Single index table consumed by nof_pack_mlp: frags then biases."""
    ft, base = frag_table(n_in, ff)
    bt = bias_table(n_in, ff)
    return np.concatenate([ft.reshape(-1), bt.reshape(-1)]).astype(np.int32), base, ft.shape[0]


EXPECTED_BASE = {"L1": 0, "L2": 4, "L3": 8, "L4": 12, "L5": 20, "B5": 24, "B4": 26, "B3": 34, "B2": 38, "B1": 42}
N_FRAGS = 46
