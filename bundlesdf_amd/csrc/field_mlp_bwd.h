// The MLP backward kernels of the fused field step: k_mlp_bwd (fp32 / generic) and k_mlp_bwd_tr
// (amp, LDS transposes), with their weight-gradient flushes. Not a standalone header: field_step.hip
// includes it inside namespace nof, after the forward kernels whose helpers (FieldArgs, the MFMA
// fragment helpers, the tile records, bwd_entry) it uses.
#pragma once

// ---------------------------------------------- kernel 3: MLP backward + dW
// Persistent waves (one per SIMD) over the tiles k_encode flagged (k_compact's
// list). Per tile (32 samples) the forward is recomputed from the encoded
// features, the loss gradient of each sample is formed from k_encode's per-sample
// terms and the ray's dL/drgb (raw2outputs backward), and the backward runs on
// MFMA — and every weight / bias gradient of the tile is added to accumulators
// the wave keeps in registers across all of its tiles (written once, at the end).
//
// Two layouts of each activation: "normal" (lane = sample, the layer chain's B
// operand) and "transposed" (lane = unit, accumulator registers = samples),
// obtained with the operands swapped: mma(acc, act, W) with the SAME weight
// fragments computes act^T W^T. The transposed accumulators of a layer's input
// (X^t) and of its output gradient (dY^t) pair the samples of their registers
// identically, so mma(dW, frag(dY^t), frag(X^t)) is dW += dY X^T with
// K = the tile's samples: no LDS transposes and no tile records in HBM.
// Writes dL/dfeature chunks (scaled; k_scatter) and, for weighted tiles, the
// view-direction part of dL/dtf (through the SH encoding) into the ray's pose
// gradient and the frame-feature gradient.
template <typename TM>
__device__ __forceinline__ typename FragT<TM>::T id_acc_frag(int s, int lane) {
    // identity B operand for acc-ordered rows: element j of K step s is row 16s + 8(j>>2) + 4h + (j&3)
    const int n = lane & 31, h = lane >> 5;
    typename FragT<TM>::T f;
#pragma unroll
    for (int j = 0; j < 8; ++j) frag_set<TM>(f, j, (16 * s + 8 * (j >> 2) + 4 * h + (j & 3)) == n ? 1.f : 0.f);
    return f;
}
template <typename TM>
__device__ __forceinline__ typename FragT<TM>::T id_nat_frag(int lane) {   // natural K order 8h + j (dO)
    const int n = lane & 31, h = lane >> 5;
    typename FragT<TM>::T f;
#pragma unroll
    for (int j = 0; j < 8; ++j) frag_set<TM>(f, j, (8 * h + j) == n ? 1.f : 0.f);
    return f;
}
// transposed activation: + per-lane (unit) bias, optional ReLU, rounded to TM, as K =
// samples fragments; returns the ReLU mask of the lane's unit (bit q: register q > 0)
template <typename TM>
__device__ __forceinline__ uint32_t tr_finish(f16v &acc, float bias, bool relu, typename FragT<TM>::T (&f)[2]) {
    uint32_t m = 0;
    if constexpr (sizeof(TM) == 2) {
#pragma unroll
        for (int p = 0; p < 8; ++p) {
            h2v u = pk_round(acc[2 * p] + bias, acc[2 * p + 1] + bias);
            if (relu) {
                u = relu_pk(u);
                m |= pair_bits(u, p);
            }
            frag_put2(f[p >> 2], p & 3, u);
        }
    } else {
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            float v = acc[q] + bias;
            if (relu) v = fmaxf(v, 0.f);
            acc[q] = v;
            m |= (v > 0.f ? 1u : 0u) << q;
        }
        acc_to_frag<TM>(acc, 0, false, f[0]);
        acc_to_frag<TM>(acc, 1, false, f[1]);
    }
    return m;
}
// transposed gradient: ReLU mask bits of the unit's activation, per-lane bias sum,
// K = samples fragments
template <typename TM>
__device__ __forceinline__ void tr_grad(f16v &acc, uint32_t mask, float &bsum, typename FragT<TM>::T (&f)[2]) {
    if constexpr (sizeof(TM) == 2) {
        // packed: round the pair, mask it, and add both halves to the bias sum with one
        // v_dot2_f32_f16 (fp32 accumulation of the rounded fp16 gradients)
#pragma unroll
        for (int p = 0; p < 8; ++p) {
            const h2v u = pk_keep(pk_round(acc[2 * p], acc[2 * p + 1]), mask, p);
            bsum = __builtin_amdgcn_fdot2(u, h2v{(_Float16)1.f, (_Float16)1.f}, bsum, false);
            frag_put2(f[p >> 2], p & 3, u);
        }
    } else {
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const float v = ((mask >> q) & 1u) ? acc[q] : 0.f;
            acc[q] = v;
            bsum += v;
        }
        acc_to_frag<TM>(acc, 0, false, f[0]);
        acc_to_frag<TM>(acc, 1, false, f[1]);
    }
}
template <typename TM>
__device__ __forceinline__ void dw_add(f16v &dw, const typename FragT<TM>::T (&dy)[2], const typename FragT<TM>::T (&x)[2]) {
    mma(dw, dy[0], x[0]);
    mma(dw, dy[1], x[1]);
}

// ---- a wave's weight / bias gradients at the end of k_mlp_bwd: one atomic per element (lanes =
// consecutive columns). dwa: PASS 0 dW4 (ot * 2 + it), dW5 (4 + it); PASS 1 dW1 (ot), dW2 (2 + it),
// dW3 (4 + ot); dba: partial bias sums of the lane's unit (both lane halves, combined here)
template <typename TM, int PASS>
__device__ __forceinline__ void mlp_bwd_flush(const FieldArgs &a, f16v (&dwa)[6], float (&dba)[5], int n, int h) {
    const MlpOff mo(a.mlp_in, a.n_ff);
    float *grad = a.grad_mlp;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        const int row = acc_row(q, h);
        if constexpr (PASS == 0) {
#pragma unroll
            for (int ot = 0; ot < 2; ++ot)
#pragma unroll
                for (int it = 0; it < 2; ++it)
                    atomic_add_f32(grad + mo.w4 + (32 * ot + row) * 64 + 32 * it + n, dwa[ot * 2 + it][q]);
#pragma unroll
            for (int t = 0; t < 2; ++t)
                if (row < 3) atomic_add_f32(grad + mo.w5 + row * 64 + 32 * t + n, dwa[4 + t][q]);
        } else {
            const int col = cin_col(n, a.n_ff);
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                if (n < mo.in) atomic_add_f32(grad + mo.w1 + (32 * t + row) * mo.in + n, dwa[t][q]);
                if (row < 16) atomic_add_f32(grad + mo.w2 + row * 64 + 32 * t + n, dwa[2 + t][q]);
                if (col >= 0) atomic_add_f32(grad + mo.w3 + (32 * t + row) * mo.cin + col, dwa[4 + t][q]);
            }
        }
    }
    // biases: lane halves hold partial sums over their samples
#pragma unroll
    for (int i = 0; i < 5; ++i) dba[i] += __shfl_xor(dba[i], 32, 64);
    if (h == 0) {
        if constexpr (PASS == 0) {
            atomic_add_f32(grad + mo.b4 + n, dba[0]);
            atomic_add_f32(grad + mo.b4 + 32 + n, dba[1]);
            if (n < 3) atomic_add_f32(grad + mo.b5 + n, dba[2]);
        } else {
            atomic_add_f32(grad + mo.b1 + n, dba[0]);
            atomic_add_f32(grad + mo.b1 + 32 + n, dba[1]);
            if (n < 16) atomic_add_f32(grad + mo.b2 + n, dba[2]);
            atomic_add_f32(grad + mo.b3 + n, dba[3]);
            atomic_add_f32(grad + mo.b3 + 32 + n, dba[4]);
        }
    }
}

// Two passes over the list split the weight-gradient accumulators (each pass
// recomputes the forward it needs): PASS 0 the colour net's last two layers
// (dW5, dW4: 6 tiles, colour tiles only); PASS 1 dW3, dW2, dW1 (6 tiles), the
// normal backward chain, dL/dfeature, the SH / frame-feature / view-direction
// gradients. ~96 accumulator registers per pass instead of 192.
// FF: frame features present (cfg frame_features > 0): their per-tile gradient sums are
// compiled only into that instance
template <typename TM, int WPB, int WAVES, int PASS, bool FF = false>
__global__ __launch_bounds__(WPB * 64) __attribute__((amdgpu_waves_per_eu(WAVES, WAVES))) void k_mlp_bwd(FieldArgs a_) {
    const FieldArgs a = step_args(a_);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int n = lane & 31, h = lane >> 5;
    typedef typename FragT<TM>::T Frag;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    stage_mlp<TM>(a, smem);
    const TM *s_fr = reinterpret_cast<const TM *>(smem);
    const float *s_b = reinterpret_cast<const float *>(smem + N_FRAGS * 64 * 8 * sizeof(TM));
    const LdsW<TM> W{s_fr};
    const float lscale = *a.loss_scale;
    const int n_c = __builtin_amdgcn_readfirstlane(a.n_tiles[0]);
    const int n_rec = PASS == 0 ? n_c : n_c + __builtin_amdgcn_readfirstlane(a.n_tiles[2]);
    const int cap = a.R * (a.S / 32);
    // weight-gradient accumulators: lane = input unit (32 it + n), registers = output rows
    //   PASS 0: dwa[0..3] = dW4 (ot * 2 + it), dwa[4..5] = dW5 (it)
    //   PASS 1: dwa[0..1] = dW1 (ot), dwa[2..3] = dW2 (it), dwa[4..5] = dW3 (ot)
    f16v dwa[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) acc_zero(dwa[i]);
    // bias-gradient partial sums of this lane's unit (both lane halves; combined at the end)
    //   PASS 0: dba[0..1] = db4, dba[2] = db5;  PASS 1: dba[0..1] = db1, dba[2] = db2, dba[3..4] = db3
    float dba[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
    float n_bwd = 0.f;
    int ff_frame = -1;     // frame-feature gradient: the frame being summed (wave-uniform), sums in s_ff
    float *s_ff = reinterpret_cast<float *>(smem + N_FRAGS * 64 * 8 * sizeof(TM) + 5 * 64 * sizeof(float)) + 4 * wave;
    const int wg = __builtin_amdgcn_readfirstlane((int)blockIdx.x * WPB + wave);
    for (int li = wg; li < n_rec; li += gridDim.x * WPB) {
        const int tsid = __builtin_amdgcn_readfirstlane(bwd_entry(a, li, n_c, cap));
        const bool colour = tsid >= 0;
        const int sid0 = tsid & 0x7fffffff;
        const size_t slot = (size_t)(sid0 >> 5);
        const int r = sid0 / a.S;
        const size_t sid = (size_t)sid0 + n;
        Frag X[2];
        if constexpr (PASS == 1) {
            X[0] = load_chunk<TM>(a.feat, (size_t)sid0, n, 0, h);
            X[1] = load_chunk<TM>(a.feat, (size_t)sid0, n, 1, h);
        }
        const float *ra = a.ray_aux + (size_t)r * RAY_AUX;
        const float4 sd = a.tile_aux[slot * TILE_AUX + 64 + n];
        const float rw = ra[4];
        const float dsdf = sd.x * rw * lscale;
        const bool valid = sd.z != 0.f;
        if (PASS == 1 && h == 0) n_bwd += sd.z;
        // ---- forward: normal (the layer chain) and, where a weight gradient needs it, transposed
        Acts<TM> A;
        f16v acc[2];
        uint32_t m1 = 0u;
        if constexpr (PASS == 1) {   // (pass 0 starts at the colour net: k_encode's Cin[0])
#pragma unroll
            for (int mt = 0; mt < 2; ++mt) {
                acc_init_bias(acc[mt], s_b + 0 * 64, mt, h);
#pragma unroll
                for (int s = 0; s < 2; ++s) mma(acc[mt], W.get(FR_L1 + mt * 2 + s, lane), X[s]);
            }
#pragma unroll
            for (int t = 0; t < 2; ++t)
#pragma unroll
                for (int s = 0; s < 2; ++s) acc_to_frag<TM>(acc[t], s, true, A.H1[t][s]);
            m1 = relu_mask<TM>(A.H1);
        }
        Frag dH2;                  // normal dL/d(sigma-net output), K step 0 (rows 0..15)
        f16v dt[2];                // transposed gradient accumulators
        if (colour) {
            const RayCtx c = load_ray(a, r);
            Frag dO;
            frag_zero<TM>(dO);
            uint32_t m3, m4, m3t[2];
            Frag Cint[2];
            if constexpr (PASS == 0) {
            // colour-net input: rows 0..15 (sdf, geo) as k_encode formed them (the same bits
            // the L1 / L2 recompute would give); rows 16.. the ray's SH / frame features
            A.Cin[0] = load_cin<TM>(a.tile_aux + slot * TILE_AUX, lane);
            A.Cin[1] = sh_frag<TM>(c, h, a.n_ff);
            // L3, normal and transposed (dW4's input, the transposed ReLU mask for pass 1's dH3^t)
            Frag H3t[2][2];
#pragma unroll
            for (int mt = 0; mt < 2; ++mt) {
                acc_init_bias(acc[mt], s_b + 2 * 64, mt, h);
                f16v ht;
                acc_zero(ht);
#pragma unroll
                for (int s = 0; s < 2; ++s) {
                    const Frag w = W.get(FR_L3 + mt * 2 + s, lane);
                    mma(acc[mt], w, A.Cin[s]);
                    mma(ht, A.Cin[s], w);
                }
                m3t[mt] = tr_finish<TM>(ht, s_b[2 * 64 + 32 * mt + n], true, H3t[mt]);
            }
#pragma unroll
            for (int t = 0; t < 2; ++t)
#pragma unroll
                for (int s = 0; s < 2; ++s) acc_to_frag<TM>(acc[t], s, true, A.H3[t][s]);
            m3 = relu_mask<TM>(A.H3);
            // hand-off to pass 1 (which then skips the L3..L5 forward), each part stored when it
            // is formed: the ReLU masks of H3 / H3^t here, of H4 and dO below
            {
                const uint32_t m3tp = (sizeof(TM) == 2) ? (m3t[0] | (m3t[1] << 8)) : (m3t[0] | (m3t[1] << 16));
                *reinterpret_cast<uint2 *>(a.tile_aux + slot * TILE_AUX + lane) = make_uint2(m3, m3tp);
            }
            // L4, normal and transposed (dW5's input and the ReLU mask of dH4^t)
            uint32_t m4t[2];
            Frag H4t[2][2];
#pragma unroll
            for (int mt = 0; mt < 2; ++mt) {
                acc_init_bias(acc[mt], s_b + 3 * 64, mt, h);
                f16v ht;
                acc_zero(ht);
#pragma unroll
                for (int t = 0; t < 2; ++t)
#pragma unroll
                    for (int s = 0; s < 2; ++s) {
                        const Frag w = W.get(FR_L4 + mt * 4 + 2 * t + s, lane);
                        mma(acc[mt], w, A.H3[t][s]);
                        mma(ht, A.H3[t][s], w);
                    }
                m4t[mt] = tr_finish<TM>(ht, s_b[3 * 64 + 32 * mt + n], true, H4t[mt]);
            }
#pragma unroll
            for (int t = 0; t < 2; ++t)
#pragma unroll
                for (int s = 0; s < 2; ++s) acc_to_frag<TM>(acc[t], s, true, A.H4[t][s]);
            m4 = relu_mask<TM>(A.H4);
            reinterpret_cast<uint32_t *>(a.tile_aux + slot * TILE_AUX + lane)[2] = m4;
            // L5 -> logits (rows 0..2, half 0)
            acc_init_bias(acc[0], s_b + 4 * 64, 0, h);
#pragma unroll
            for (int t = 0; t < 2; ++t)
#pragma unroll
                for (int s = 0; s < 2; ++s) mma(acc[0], W.get(FR_L5 + 2 * t + s, lane), A.H4[t][s]);
            float logit[3];
#pragma unroll
            for (int cc = 0; cc < 3; ++cc) {
                float v = acc[0][cc];
                if constexpr (sizeof(TM) == 2) v = (float)(_Float16)v;
                logit[cc] = __shfl(v, n, 64);
            }
            // ---- loss gradient at the logits (raw2outputs backward + fs_rgb)
            const float wn = sd.y / (ra[3] + 1e-10f);
            const float gfr = a.fs_rgb_w * 2.f * sd.w * rw * a.inv_3RS;
            float gl[3];
#pragma unroll
            for (int cc = 0; cc < 3; ++cc) {
                const float sg = sigmoidf(logit[cc]);
                gl[cc] = (ra[cc] * wn + gfr * (sg - 1.f)) * sg * (1.f - sg) * lscale;
            }
            if (h == 0) {
#pragma unroll
                for (int cc = 0; cc < 3; ++cc) frag_set<TM>(dO, cc, gl[cc]);
            }
            if (h == 0) a.tile_aux[slot * TILE_AUX + 96 + n] = make_float4(gl[0], gl[1], gl[2], 0.f);
            // dW5 += dO H4^T, db5; dH4^t -> dW4 += dH4 H3^T, db4
            f16v dot;
            acc_zero(dot);
            mma(dot, dO, id_nat_frag<TM>(lane));
            Frag dOt[2];
            tr_grad<TM>(dot, MASK_ALL, dba[2], dOt);
            dw_add<TM>(dwa[4], dOt, H4t[0]);
            dw_add<TM>(dwa[5], dOt, H4t[1]);
#pragma unroll
            for (int mt = 0; mt < 2; ++mt) {
                acc_zero(dt[mt]);
                mma(dt[mt], dO, W.get(FR_B5 + mt, lane));
                Frag dH4t[2];
                tr_grad<TM>(dt[mt], m4t[mt], dba[mt], dH4t);
                dw_add<TM>(dwa[mt * 2 + 0], dH4t, H3t[0]);
                dw_add<TM>(dwa[mt * 2 + 1], dH4t, H3t[1]);
            }
            continue;
            } else {
                // Cin^t (dW3's input): L2 transposed (rows 0..15); rows 16.. are the ray's SH /
                // frame features, the same for every sample. The L3..L5 forward is not
                // recomputed: pass 0 handed over the ReLU masks and dO.
                f16v cint;
                acc_zero(cint);
#pragma unroll
                for (int t = 0; t < 2; ++t)
#pragma unroll
                    for (int s = 0; s < 2; ++s) mma(cint, A.H1[t][s], W.get(FR_L2 + 2 * t + s, lane));
                {
                    float shv[9];
                    sh_values(c, shv);
                    float crow = 0.f;   // Cin^t value of rows >= 16 (constant over samples)
                    if (n >= 16 && n <= 24) crow = shv[n - 16];
                    else if (n >= 25 && n < 25 + a.n_ff) crow = a.ff[(size_t)c.frame * a.n_ff + (n - 25)];
                    if constexpr (sizeof(TM) == 2) crow = (float)(_Float16)crow;
#pragma unroll
                    for (int q = 0; q < 16; ++q) cint[q] = (n < 16) ? cint[q] : 0.f;
                    tr_finish<TM>(cint, n < 16 ? s_b[1 * 64 + n] : crow, false, Cint);
                }
                const uint4 hm = reinterpret_cast<const uint4 *>(a.tile_aux)[slot * TILE_AUX + lane];
                m3 = hm.x;
                m4 = hm.z;
                m3t[0] = (sizeof(TM) == 2) ? (hm.y & 0x00ff00ffu) : (hm.y & 0xffffu);
                m3t[1] = (sizeof(TM) == 2) ? ((hm.y >> 8) & 0x00ff00ffu) : (hm.y >> 16);
                if (h == 0) {
                    const float4 gl = a.tile_aux[slot * TILE_AUX + 96 + n];
                    frag_set<TM>(dO, 0, gl.x);
                    frag_set<TM>(dO, 1, gl.y);
                    frag_set<TM>(dO, 2, gl.z);
                }
                // ---- L5 / L4 backward, normal chain: dH4, dH3 (+ transposed dH3 for dW3)
                Frag dH[2][2];
#pragma unroll
                for (int mt = 0; mt < 2; ++mt) {
                    acc_zero(acc[mt]);
                    mma(acc[mt], W.get(FR_B5 + mt, lane), dO);
                }
                masked_frags<TM>(acc, m4, dH);
                // dH3^t -> dW3 += dH3 Cin^T, db3 first, one transposed accumulator at a time
#pragma unroll
                for (int mt = 0; mt < 2; ++mt) {
                    acc_zero(dt[0]);
#pragma unroll
                    for (int t2 = 0; t2 < 2; ++t2)
#pragma unroll
                        for (int s2 = 0; s2 < 2; ++s2) mma(dt[0], dH[t2][s2], W.get(FR_B4 + mt * 4 + 2 * t2 + s2, lane));
                    Frag dH3t[2];
                    tr_grad<TM>(dt[0], m3t[mt], dba[3 + mt], dH3t);
                    dw_add<TM>(dwa[4 + mt], dH3t, Cint);
                }
                // then the normal chain dH3
#pragma unroll
                for (int mt = 0; mt < 2; ++mt) {
                    acc_zero(acc[mt]);
#pragma unroll
                    for (int t2 = 0; t2 < 2; ++t2)
#pragma unroll
                        for (int s2 = 0; s2 < 2; ++s2) mma(acc[mt], W.get(FR_B4 + mt * 4 + 2 * t2 + s2, lane), dH[t2][s2]);
                }
                masked_frags<TM>(acc, m3, dH);
                // ---- L3 backward: dCin (the chain, SH / feature gradients)
                acc_zero(acc[0]);
#pragma unroll
                for (int t2 = 0; t2 < 2; ++t2)
#pragma unroll
                    for (int s2 = 0; s2 < 2; ++s2) mma(acc[0], W.get(FR_B3 + 2 * t2 + s2, lane), dH[t2][s2]);
                // dL/dSH of the tile (h0 rows: SH0..3, SH8; h1: SH4..7) -> view-direction part of
                // dL/dtf[:3,:3] (input_dirs = R vd, run_network :1281), added to the ray's pose gradient
                if (FF && a.n_ff > 0) {   // dL/d frame features = sum over the tile of dCin rows 25.. (h0: acc 13..15)
                    const float d0 = wave_sum(h == 0 ? acc[0][13] : 0.f);
                    const float d1 = a.n_ff > 1 ? wave_sum(h == 0 ? acc[0][14] : 0.f) : 0.f;
                    const float d2 = a.n_ff > 2 ? wave_sum(h == 0 ? acc[0][15] : 0.f) : 0.f;
                    // summed in registers while the wave's tiles stay on one frame (the list is
                    // frame-major), one atomic per frame change: F x n_ff words on a few cache
                    // lines would otherwise take an atomic from every tile
                    // (the running sums live in the wave's LDS words, not in registers)
                    if (lane < a.n_ff) {
                        const float dv = lane == 0 ? d0 : (lane == 1 ? d1 : d2);
                        if (c.frame != ff_frame) {
                            if (ff_frame >= 0 && !ABL(512))   // ABL 512 (timing build): no frame-feature atomics
                                atomic_add_f32(a.grad_ff + (size_t)ff_frame * a.n_ff + lane, s_ff[lane]);
                            s_ff[lane] = dv;
                        } else {
                            s_ff[lane] += dv;
                        }
                    }
                    ff_frame = c.frame;
                }
                if (!a.no_dx) {
                    float g[9];
                    float unused;
                    half_sums(acc[0][8], g[0], g[4]);
                    half_sums(acc[0][9], g[1], g[5]);
                    half_sums(acc[0][10], g[2], g[6]);
                    half_sums(acc[0][11], g[3], g[7]);
                    half_sums(acc[0][12], g[8], unused);
                    const float x = (c.Rm[0][0] * c.vd[0] + c.Rm[0][1] * c.vd[1]) + c.Rm[0][2] * c.vd[2];
                    const float y = (c.Rm[1][0] * c.vd[0] + c.Rm[1][1] * c.vd[1]) + c.Rm[1][2] * c.vd[2];
                    const float zz = (c.Rm[2][0] * c.vd[0] + c.Rm[2][1] * c.vd[1]) + c.Rm[2][2] * c.vd[2];
                    const float gdir[3] = {
                        -SH_C1 * g[3] + SH_C2_0 * y * g[4] + SH_C2_2 * (-2.f * x) * g[6] + SH_C2_3 * zz * g[7] +
                            SH_C2_4 * 2.f * x * g[8],
                        -SH_C1 * g[1] + SH_C2_0 * x * g[4] + SH_C2_1 * zz * g[5] + SH_C2_2 * (-2.f * y) * g[6] -
                            SH_C2_4 * 2.f * y * g[8],
                        SH_C1 * g[2] + SH_C2_1 * y * g[5] + SH_C2_2 * 4.f * zz * g[6] + SH_C2_3 * x * g[7]};
                    const int i = (lane >> 2) % 3, j = lane & 3;
                    const float gi = i == 0 ? gdir[0] : (i == 1 ? gdir[1] : gdir[2]);
                    const float vj = j == 0 ? c.vd[0] : (j == 1 ? c.vd[1] : c.vd[2]);
                    if (lane < 12 && j < 3) atomic_add_f32(a.ray_grad + (size_t)r * 12 + lane, gi * vj);
                }
                acc_to_frag<TM>(acc[0], 0, false, dH2);
            }
        } else {
            // sigma-net-only tile: the only output gradient is dsdf (row 0)
            frag_zero<TM>(dH2);
        }
        if constexpr (PASS == 1) {
            if (h == 0) frag_set<TM>(dH2, 0, dsdf);
            // H1^t (dW2's input, and the transposed ReLU mask of dH1^t) and X^t (dW1's input),
            // formed only now from the re-read features so they are not live across the chain
            uint32_t m1t[2];
            Frag H1t[2][2], Xt[2];
            {
                Frag Xr[2];
                Xr[0] = load_chunk<TM>(a.feat, (size_t)sid0, n, 0, h);
                Xr[1] = load_chunk<TM>(a.feat, (size_t)sid0, n, 1, h);
#pragma unroll
                for (int mt = 0; mt < 2; ++mt) {
                    f16v ht;
                    acc_zero(ht);
#pragma unroll
                    for (int s = 0; s < 2; ++s) mma(ht, Xr[s], W.get(FR_L1 + mt * 2 + s, lane));
                    m1t[mt] = tr_finish<TM>(ht, s_b[0 * 64 + 32 * mt + n], true, H1t[mt]);
                }
                f16v xt;
                acc_zero(xt);
                mma(xt, Xr[0], id_acc_frag<TM>(0, lane));
                mma(xt, Xr[1], id_acc_frag<TM>(1, lane));
                acc_to_frag<TM>(xt, 0, false, Xt[0]);
                acc_to_frag<TM>(xt, 1, false, Xt[1]);
            }
            // ---- L2 backward: dW2 / db2 from dH2^t (an identity transpose of the normal
            // fragment: rows 1..15 dCin geo, row 0 dsdf), dH1 (normal + transposed)
            {
                acc_zero(dt[0]);
                mma(dt[0], dH2, id_acc_frag<TM>(0, lane));
                Frag dH2t[2];
                tr_grad<TM>(dt[0], MASK_ALL, dba[2], dH2t);
                dw_add<TM>(dwa[2], dH2t, H1t[0]);
                dw_add<TM>(dwa[3], dH2t, H1t[1]);
            }
            Frag dH1[2][2];
#pragma unroll
            for (int mt = 0; mt < 2; ++mt) {
                acc_zero(acc[mt]);
                acc_zero(dt[mt]);
                const Frag w = W.get(FR_B2 + mt * 2, lane);
                mma(acc[mt], w, dH2);
                mma(dt[mt], dH2, w);
            }
            masked_frags<TM>(acc, m1, dH1);
#pragma unroll
            for (int mt = 0; mt < 2; ++mt) {
                Frag dH1t[2];
                tr_grad<TM>(dt[mt], m1t[mt], dba[mt], dH1t);
                dw_add<TM>(dwa[mt], dH1t, Xt);
            }
            // ---- L1 backward: dX = W1^T dH1 -> feature gradients in this lane's level order
            acc_zero(acc[0]);
#pragma unroll
            for (int t2 = 0; t2 < 2; ++t2)
#pragma unroll
                for (int s2 = 0; s2 < 2; ++s2) mma(acc[0], W.get(FR_B1 + 2 * t2 + s2, lane), dH1[t2][s2]);
#pragma unroll
            for (int ss = 0; ss < 2; ++ss) {
                Frag f;
#pragma unroll
                for (int j = 0; j < 8; ++j) frag_set<TM>(f, j, valid ? acc[0][8 * ss + j] : 0.f);
                store_dfeat<TM>(a.dfeat, (size_t)a.R * a.S, (size_t)sid0, n, ss, h, f);
            }
        }
    }
    if constexpr (PASS == 1) {
        n_bwd = wave_sum(n_bwd);
        if (lane == 0) atomic_add_f32(loss_row(a, wg) + 5, n_bwd);
        if (FF && ff_frame >= 0 && lane < a.n_ff) atomic_add_f32(a.grad_ff + (size_t)ff_frame * a.n_ff + lane, s_ff[lane]);
    }
    if (wg >= n_rec || ABL(1 << 21)) return;
    mlp_bwd_flush<TM, PASS>(a, dwa, dba, n, h);
}

// ------------------------------- kernel 3 (amp): MLP backward with LDS transposes
// The fp16 (amp) form of k_mlp_bwd: two passes over k_compact's tile list with the same outputs
// (dW / db accumulated in registers over the wave's tiles, one atomic per element at the end;
// dL/dfeature; the SH / frame-feature / view-direction gradients), but every weight gradient
// takes its K = samples operands from LDS: each activation and each masked gradient of the
// normal chain is written once into a per-wave [32 samples][32 units] image and read back
// transposed (mlp_lds.h: ds_read_b64_tr_b16); the transposed values are bit-identical to the
// normal ones. The passes split at the sigma net's output (k_mlp_bwd_tr below).
// The amp weight-gradient accumulators and bias sums of one pass, flushed per wave (one atomic per
// element) or summed over the block first. PASS 0 (colour): dW4 (f = ot * 2 + it), dW5 (4, the
// 16x16 layout of dw16_tr), dW3 (5 + ot); biases b4 (0, 1), b5 (2, dw16_tr's lane groups), b3 (3, 4).
// PASS 1 (sigma): dW1 (ot), dW2 (2, 16x16 layout); biases b1 (0, 1), b2 (2, lane groups).
// Fragment f, element (q, lane) -> parameter:
template <int PASS>
__device__ __forceinline__ void amp_dw_atomic(const FieldArgs &a, const MlpOff &mo, int f, int q, int ln, float v) {
    const int n = ln & 31, row = acc_row(q, ln >> 5), t = f & 1;
    // dw16_tr's element q = 4 b + j: out unit 4 (lane >> 4) + j, in unit 16 b + (lane & 15)
    const int row16 = 4 * (ln >> 4) + (q & 3), col16 = 16 * (q >> 2) + (ln & 15);
    float *grad = a.grad_mlp;
    if constexpr (PASS == 0) {
        if (f < 4) {
            atomic_add_f32(grad + mo.w4 + (32 * (f >> 1) + row) * 64 + 32 * t + n, v);
        } else if (f == 4) {
            if (row16 < 3) atomic_add_f32(grad + mo.w5 + row16 * 64 + col16, v);
        } else {
            const int col = cin_col(n, a.n_ff);
            if (col >= 0) atomic_add_f32(grad + mo.w3 + (32 * (f - 5) + row) * mo.cin + col, v);
        }
    } else {
        if (f < 2) {
            if (n < mo.in) atomic_add_f32(grad + mo.w1 + (32 * t + row) * mo.in + n, v);
        } else {
            atomic_add_f32(grad + mo.w2 + row16 * 64 + col16, v);
        }
    }
}
template <int PASS>
__device__ __forceinline__ float *amp_db_dst(const FieldArgs &a, const MlpOff &mo, int i, int n) {
    float *grad = a.grad_mlp;
    if constexpr (PASS == 0) {
        return i == 0 ? grad + mo.b4 + n
                      : (i == 1 ? grad + mo.b4 + 32 + n
                                : (i == 2 ? (n < 3 ? grad + mo.b5 + n : nullptr) : grad + mo.b3 + 32 * (i - 3) + n));
    } else {
        return i == 0 ? grad + mo.b1 + n : (i == 1 ? grad + mo.b1 + 32 + n : (n < 16 ? grad + mo.b2 + n : nullptr));
    }
}
template <int PASS, int NF, int NB>
__device__ __forceinline__ void amp_bwd_flush(const FieldArgs &a, f16v (&dwa)[NF], float (&dba)[NB], int lane) {
    const MlpOff mo(a.mlp_in, a.n_ff);
#pragma unroll
    for (int f = 0; f < NF; ++f)
#pragma unroll
        for (int q = 0; q < 16; ++q) amp_dw_atomic<PASS>(a, mo, f, q, lane, dwa[f][q]);
#pragma unroll
    for (int i = 0; i < NB; ++i) dba[i] += __shfl_xor(dba[i], 32, 64);   // both lane halves' partial sums
    if (lane < 32) {
#pragma unroll
        for (int i = 0; i < NB; ++i) {
            float *d = amp_db_dst<PASS>(a, mo, i, lane);
            if (d) atomic_add_f32(d, dba[i]);
        }
    }
}
// summed over the block in LDS first (FPR fragments per LDS round), one atomic per non-zero element
template <int PASS, int NF, int NB, int FPR>
__device__ __forceinline__ void amp_bwd_flush_block(const FieldArgs &a, f16v (&dwa)[NF], float (&dba)[NB], char *smem,
                                                    int wave, int lane, int nw) {
    const MlpOff mo(a.mlp_in, a.n_ff);
    float *buf = reinterpret_cast<float *>(smem);
    const int tid = threadIdx.x, nthr = blockDim.x;
#pragma unroll
    for (int i = 0; i < NB; ++i) dba[i] += __shfl_xor(dba[i], 32, 64);
    __syncthreads();   // every wave is past its tiles: weights, biases and images are free
    if (lane < 32) {
#pragma unroll
        for (int i = 0; i < NB; ++i) buf[(wave * NB + i) * 32 + lane] = dba[i];
    }
    __syncthreads();
    if (tid < NB * 32) {
        const int i = tid >> 5, n = tid & 31;
        float v = 0.f;
        for (int w = 0; w < nw; ++w) v += buf[(w * NB + i) * 32 + n];
        float *d = amp_db_dst<PASS>(a, mo, i, n);
        if (d && v != 0.f) atomic_add_f32(d, v);
    }
    __syncthreads();
#pragma unroll
    for (int f0 = 0; f0 < NF; f0 += FPR) {
#pragma unroll
        for (int j = 0; j < FPR; ++j)
            if (f0 + j < NF) {
#pragma unroll
                for (int q = 0; q < 16; ++q) buf[((j * nw + wave) * 16 + q) * 64 + lane] = dwa[f0 + j][q];
            }
        __syncthreads();
        const int nf = min(FPR, NF - f0);
        for (int e = tid; e < nf * 1024; e += nthr) {
            const int j = e >> 10, q = (e >> 6) & 15, ln = e & 63;
            float v = 0.f;
            for (int w = 0; w < nw; ++w) v += buf[((j * nw + w) * 16 + q) * 64 + ln];
            if (v != 0.f) amp_dw_atomic<PASS>(a, mo, f0 + j, q, ln, v);
        }
        __syncthreads();
    }
}

// LDS of one k_mlp_bwd_tr block. PASS 0: all weight fragments, biases, 4 frame-feature floats per
// wave, then 6 images per wave. PASS 1: only the fragments it reads (L1, B2, B1: 12 KB) and b1, then
// 4 images per wave
constexpr int BWD_IMGS0 = 6, BWD_IMGS1 = 4;
constexpr int S1_NFR = 12;   // PASS 1's fragments: FR_L1 .. FR_L1 + 3, FR_B2 .. FR_B1 + 3
__host__ __device__ constexpr size_t bwd_tr_img_base(int pass, int wpb) {
    return pass == 0 ? (((size_t)N_FRAGS * 64 * 8 * 2 + 5 * 64 * 4 + 16 * (size_t)wpb + 15) & ~(size_t)15)
                     : (size_t)S1_NFR * 64 * 8 * 2 + 64 * 4;
}
__host__ __device__ constexpr size_t bwd_tr_lds(int pass, int wpb) {
    return bwd_tr_img_base(pass, wpb) + (size_t)wpb * (pass == 0 ? BWD_IMGS0 : BWD_IMGS1) * IMG_BYTES;
}
// PASS 1's fragment accessor: FR_L1 .. FR_L1 + 3 at LDS slots 0..3, FR_B2 .. FR_B1 + 3 at 4..11
struct LdsW1 {
    const _Float16 *p;
    __device__ __forceinline__ h8v get(int f, int lane) const {
        const int s = f < FR_L2 ? f : f - FR_B2 + 4;
        return reinterpret_cast<const h8v *>(p)[s * 64 + lane];
    }
};
__device__ __forceinline__ void stage_sigma_bwd(const FieldArgs &a, char *smem) {
    const uint4 *src = reinterpret_cast<const uint4 *>(a.frags);
    uint4 *dst = reinterpret_cast<uint4 *>(smem);
    constexpr int per = 64 * 8 * 2 / 16;   // 16-B pieces per fragment
    for (int i = threadIdx.x; i < S1_NFR * per; i += blockDim.x) {
        const int f = i / per, sf = f < 4 ? FR_L1 + f : FR_B2 + (f - 4);
        dst[i] = src[sf * per + (i - f * per)];
    }
    float *s_b = reinterpret_cast<float *>(smem + S1_NFR * 64 * 8 * 2);
    for (int i = threadIdx.x; i < 64; i += blockDim.x) s_b[i] = a.bias[i];
    __syncthreads();
}
__device__ __forceinline__ void lds_wave_sync() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); }

// bias-gradient partial sum of one transposed gradient fragment (this lane's unit, 8 samples)
__device__ __forceinline__ float frag_sum(const h8v &f, float acc) {
#pragma unroll
    for (int p = 0; p < 4; ++p)
        acc = __builtin_amdgcn_fdot2(h2v{f[2 * p], f[2 * p + 1]}, h2v{(_Float16)1.f, (_Float16)1.f}, acc, false);
    return acc;
}
// dW += A^T B over the tile's 32 samples: A, B images of [32 samples][32 units] (out / in units)
__device__ __forceinline__ void dw_tr(f16v &dw, const char *imgA, const char *imgB, int lane, float *bsum) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
        const h8v a = img_read_tr(imgA, ks, lane);
        if (bsum) *bsum = frag_sum(a, *bsum);
        mma(dw, a, img_read_tr(imgB, ks, lane));
    }
}
// dW (16 out units x 64 in units) += A^T B over the tile's 32 samples as four 16x16x32 MFMAs — half
// the MFMA cycles and accumulator registers of two 32x32 blocks whose out rows 16..31 are padding
// (dW2: 16 out units, dW5: 3). A: image of [32 samples][out units 0..15 (of 32)]; B0, B1: the in
// units' two 32-unit images. dw element 4 b + j = (out 4 (lane >> 4) + j, in 16 b + (lane & 15));
// bsum: this lane's partial of out unit lane & 15 (the four lane groups summed at the flush)
__device__ __forceinline__ void dw16_tr(f16v &dw, const char *imgA, const char *imgB0, const char *imgB1, int lane,
                                        float *bsum) {
    typedef float f4v __attribute__((ext_vector_type(4)));
    const h8v a = img_read_tr_k32(imgA, 0, lane);
    if (bsum) *bsum = frag_sum(a, *bsum);
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        const h8v x = img_read_tr_k32(b < 2 ? imgB0 : imgB1, b & 1, lane);
        f4v c = {dw[4 * b], dw[4 * b + 1], dw[4 * b + 2], dw[4 * b + 3]};
        c = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, x, c, 0, 0, 0);
#pragma unroll
        for (int j = 0; j < 4; ++j) dw[4 * b + j] = c[j];
    }
}

// The amp MLP backward in two passes split at the sigma net's output (the colour net's input):
//   PASS 0 (colour-backward tiles, the list's front): L3, L4, L5 forward from the colour-net input
//     (k_encode), the logit gradient dO, dW5 += dO^T H4, dH4, dW4 += dH4^T H3, dH3, dW3 += dH3^T Cin,
//     dCin = B3 dH3 (SH / frame-feature / view-direction pose gradients); hands pass 1 the sigma-net
//     output gradient dCin rows 0..15 through the tile aux (the colour-net input's slot, consumed).
//     dW3 / dW4 / dW5: 8 accumulator fragments; 8-wave blocks, one per CU (2 waves / SIMD).
//   PASS 1 (every backward tile): L1 forward, dH2 (pass 0's hand-off for colour tiles, 0 for the
//     sigma-only ones, + the sdf loss gradient in row 0), dW2 += dH2^T H1, dH1, dW1 += dH1^T X,
//     dX -> dfeat. dW1 / dW2: 4 accumulator fragments, 4 LDS images, only L1 / B2 / B1 staged;
//     8-wave blocks, one per CU (2 waves / SIMD: at 3 the 168-register budget spilled 38 registers).
// (Round 4 split at the colour net's last two layers: pass 1 then held dW1..dW3 — 256 registers,
// 2 waves / SIMD — and recomputed dH4 / dH3 from the masks and dO pass 0 handed over.)
template <int WPB, int PASS, bool FF = false, bool BLK = false>
__global__ __launch_bounds__(WPB * 64) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_mlp_bwd_tr(FieldArgs a_) {
    typedef _Float16 TM;
    typedef h8v Frag;
    constexpr int NF = PASS == 0 ? 7 : 3, NB = PASS == 0 ? 5 : 3;
    const FieldArgs a = step_args(a_);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int n = lane & 31, h = lane >> 5;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    if constexpr (PASS == 0) stage_mlp<TM>(a, smem);
    else stage_sigma_bwd(a, smem);
    const TM *s_fr = reinterpret_cast<const TM *>(smem);
    const float *s_b = reinterpret_cast<const float *>(smem + (PASS == 0 ? N_FRAGS : S1_NFR) * 64 * 8 * sizeof(TM));
    float *s_ff = const_cast<float *>(s_b) + 5 * 64 + 4 * wave;   // PASS 0 (FF) only
    char *img = smem + bwd_tr_img_base(PASS, WPB) + (size_t)wave * (PASS == 0 ? BWD_IMGS0 : BWD_IMGS1) * IMG_BYTES;
    auto IMG = [&](int i) { return img + i * IMG_BYTES; };
    LdsWt<TM> W0(s_fr, lane);   // fenced per tile (the top of tile())
    const LdsW1 W1{s_fr};
    const float lscale = *a.loss_scale;
    // the backward list: colour-backward tiles [0, n_c) at the front, sigma-only tiles at the back
    // (k_compact); pass 0 walks the front only
    const int n_c = __builtin_amdgcn_readfirstlane(a.n_tiles[0]);
    const int n_rec = PASS == 0 ? n_c : n_c + __builtin_amdgcn_readfirstlane(a.n_tiles[2]);
    const int cap = a.R * (a.S / 32);
    f16v dwa[NF];
#pragma unroll
    for (int i = 0; i < NF; ++i) acc_zero(dwa[i]);
    float dba[NB];
#pragma unroll
    for (int i = 0; i < NB; ++i) dba[i] = 0.f;
    float n_bwd = 0.f;
    int ff_frame = -1;
    Frag zero;
    frag_zero<TM>(zero);
    const int wg = __builtin_amdgcn_readfirstlane((int)blockIdx.x * WPB + wave);
    const int stride = gridDim.x * WPB;
    // FF (frame features, PASS 0): each wave takes a contiguous run of the list instead of every
    // stride-th tile. k_compact lists each 4096-tile block of the frame-sorted batch in ray order,
    // so a run stays on one or two frames and the per-frame feature-gradient sums below leave the
    // wave a few times, not at every tile: one atomic per frame change on F x n_ff hot words
    // serialises at the memory side (config 5: 1.4 ms of k_mlp_bwd)
    int li0 = wg, lstep = stride, lend = n_rec;
    if constexpr (FF) {
        const int chunk = (n_rec + stride - 1) / stride;
        li0 = wg * chunk;
        lend = min(n_rec, li0 + chunk);
        lstep = 1;
    }
    // the tile's first operands (pass 0: the colour-net input; pass 1: the features X, pass 0's
    // hand-off) and its per-sample loss terms are loaded one tile ahead, the list entry two tiles
    // ahead, so a tile's first MFMAs do not wait for a memory latency
    int t_cur = li0 < lend ? bwd_entry(a, li0, n_c, cap) : 0;
    int t_nxt = li0 + lstep < lend ? bwd_entry(a, li0 + lstep, n_c, cap) : 0;
    Frag pre[2], dh2_n;
    pre[0] = zero;
    pre[1] = zero;
    dh2_n = zero;
    float4 sd_n = make_float4(0.f, 0.f, 0.f, 0.f);
    float rw_n = 0.f;
    auto fetch = [&](int tsid_f) {
        const int s0 = tsid_f & 0x7fffffff;
        const float4 *ax = a.tile_aux + (size_t)(s0 >> 5) * TILE_AUX;
        if constexpr (PASS == 0) {
            pre[0] = load_cin<TM>(ax, lane);
            pre[1] = reinterpret_cast<const h8v *>(ax + 192)[lane];
            sd_n = ax[64 + n];
            rw_n = a.ray_aux[(size_t)(s0 / a.S) * RAY_AUX + 4];   // the ray weight
        } else {
            pre[0] = load_chunk<TM>(a.feat, (size_t)s0, n, 0, h);
            pre[1] = load_chunk<TM>(a.feat, (size_t)s0, n, 1, h);
            sd_n = ax[64 + n];
            rw_n = a.ray_aux[(size_t)(s0 / a.S) * RAY_AUX + 4];
            dh2_n = load_cin<TM>(ax, lane);   // pass 0's hand-off (colour tiles; ignored for the others)
        }
    };
    if (li0 < lend) fetch(__builtin_amdgcn_readfirstlane(t_cur));
    auto tile = [&](auto COLT, int li) {
        if constexpr (PASS == 0) W0.fence();   // the fragment reads stay in this tile
        const int tsid = __builtin_amdgcn_readfirstlane(t_cur);
        const Frag in0 = pre[0], in1 = pre[1];
        constexpr bool colour = decltype(COLT)::value;   // the list's front: colour-backward tiles
        const int sid0 = tsid & 0x7fffffff;
        const size_t slot = (size_t)(sid0 >> 5);
        const int r = sid0 / a.S;
        const float *ra = a.ray_aux + (size_t)r * RAY_AUX;
        const float4 *aux = a.tile_aux + slot * TILE_AUX;
        // this tile's own loads go out BEFORE the next tile's prefetch: the vector-memory counter
        // retires in issue order, so waiting for them then leaves the prefetch in flight
        float dl[4] = {0.f, 0.f, 0.f, 0.f};   // pass 0: dL/drgb (x weights) and the ray's weight sum
        float2 vdw = make_float2(0.f, 0.f);   // pass 0: lanes 0..2, the ray's view directions (k_colour)
        int frame = 0;
        if constexpr (PASS == 0) {
#pragma unroll
            for (int cc = 0; cc < 4; ++cc) dl[cc] = ra[cc];
            vdw = reinterpret_cast<const float2 *>(aux + min(lane, 2))[1];
            if (FF) frame = (int)a.rays[(size_t)r * 12 + 8];
        }
        // the next tile's prefetch goes out once this tile's first layer has read the prefetched
        // operands (no copy of in-flight registers), unconditionally (the last tile re-fetches itself,
        // the entry index is clamped: a branch around these loads makes the compiler's waits conservative)
        float4 sd;
        float rw;
        Frag dh2in;
        auto advance = [&]() {
            sd = sd_n;
            rw = rw_n;
            dh2in = dh2_n;
            fetch(__builtin_amdgcn_readfirstlane(li + lstep < lend ? t_nxt : tsid));
            t_cur = t_nxt;
            t_nxt = bwd_entry(a, min(li + 2 * lstep, lend - 1), n_c, cap);
        };
        f16v acc[2];
        if constexpr (PASS == 0) {
            Frag Cin[2], H3[2][2], H4[2][2];
            Cin[0] = in0;
            Cin[1] = in1;
            // L3 (-> images 0, 1)
#pragma unroll
            for (int mt = 0; mt < 2; ++mt) {
                acc_init_bias(acc[mt], s_b + 2 * 64, mt, h);
#pragma unroll
                for (int s = 0; s < 2; ++s) mma(acc[mt], W0.get(FR_L3 + mt * 2 + s, lane), Cin[s]);
            }
            img_write(IMG(5), Cin, lane);   // dW3's B operand
            advance();   // Cin (the prefetched operands) is consumed
#pragma unroll
            for (int t = 0; t < 2; ++t)
#pragma unroll
                for (int s = 0; s < 2; ++s) acc_to_frag<TM>(acc[t], s, true, H3[t][s]);
            uint32_t r3[16];   // H3's ReLU factors, kept for dH3 below
            (void)relu_factors(H3, r3);
            img_write(IMG(0), H3[0], lane);
            img_write(IMG(1), H3[1], lane);
            // L4 (-> images 2, 3)
#pragma unroll
            for (int mt = 0; mt < 2; ++mt) {
                acc_init_bias(acc[mt], s_b + 3 * 64, mt, h);
#pragma unroll
                for (int t = 0; t < 2; ++t)
#pragma unroll
                    for (int s = 0; s < 2; ++s) mma(acc[mt], W0.get(FR_L4 + mt * 4 + 2 * t + s, lane), H3[t][s]);
            }
#pragma unroll
            for (int t = 0; t < 2; ++t)
#pragma unroll
                for (int s = 0; s < 2; ++s) acc_to_frag<TM>(acc[t], s, true, H4[t][s]);
            uint32_t r4[16];   // H4's ReLU factors, kept for dH4 below
            (void)relu_factors(H4, r4);
            img_write(IMG(2), H4[0], lane);
            img_write(IMG(3), H4[1], lane);
            // L5 -> logits (rows 0..2, half 0)
            acc_init_bias(acc[0], s_b + 4 * 64, 0, h);
#pragma unroll
            for (int t = 0; t < 2; ++t)
#pragma unroll
                for (int s = 0; s < 2; ++s) mma(acc[0], W0.get(FR_L5 + 2 * t + s, lane), H4[t][s]);
            float logit[3];
#pragma unroll
            for (int cc = 0; cc < 3; ++cc) logit[cc] = __shfl((float)(_Float16)acc[0][cc], n, 64);
            // loss gradient at the logits (raw2outputs backward + fs_rgb)
            const float wn = sd.y / (dl[3] + 1e-10f);
            const float gfr = a.fs_rgb_w * 2.f * sd.w * rw * a.inv_3RS;
            Frag dO = zero;
            if (h == 0) {
#pragma unroll
                for (int cc = 0; cc < 3; ++cc) {
                    const float sg = sigmoidf(logit[cc]);
                    frag_set<TM>(dO, cc, (dl[cc] * wn + gfr * (sg - 1.f)) * sg * (1.f - sg) * lscale);
                }
            }
            // dW5 += dO^T H4, db5 (dO image: 4, units 0..15)
            img_write1(IMG(4), dO, 0, lane);
            lds_wave_sync();
            dw16_tr(dwa[4], IMG(4), IMG(2), IMG(3), lane, &dba[2]);
            // dH4 = m4 (B5 dO) (-> images 2, 3: H4 is done), dW4 += dH4^T H3, db4
#pragma unroll
            for (int mt = 0; mt < 2; ++mt) {
                acc_zero(acc[mt]);
                mma(acc[mt], W0.get(FR_B5 + mt, lane), dO);
            }
            Frag dH[2][2];
            masked_frags_r(acc, r4, dH);
            lds_wave_sync();
            img_write(IMG(2), dH[0], lane);
            img_write(IMG(3), dH[1], lane);
            lds_wave_sync();
#pragma unroll
            for (int ot = 0; ot < 2; ++ot) {
                dw_tr(dwa[ot * 2 + 0], IMG(2 + ot), IMG(0), lane, &dba[ot]);
                dw_tr(dwa[ot * 2 + 1], IMG(2 + ot), IMG(1), lane, nullptr);
            }
            // dH3 = m3 (B4 dH4) (-> images 0, 1: H3 is done), dW3 += dH3^T Cin, db3
#pragma unroll
            for (int mt = 0; mt < 2; ++mt) {
                acc_zero(acc[mt]);
#pragma unroll
                for (int t2 = 0; t2 < 2; ++t2)
#pragma unroll
                    for (int s2 = 0; s2 < 2; ++s2) mma(acc[mt], W0.get(FR_B4 + mt * 4 + 2 * t2 + s2, lane), dH[t2][s2]);
            }
            masked_frags_r(acc, r3, dH);
            lds_wave_sync();
            img_write(IMG(0), dH[0], lane);
            img_write(IMG(1), dH[1], lane);
            lds_wave_sync();
            dw_tr(dwa[5], IMG(0), IMG(5), lane, &dba[3]);
            dw_tr(dwa[6], IMG(1), IMG(5), lane, &dba[4]);
            // dCin = B3 dH3: rows 0..15 the sigma-net output gradient (-> pass 1), 16.. SH / frame features
            acc_zero(acc[0]);
#pragma unroll
            for (int t2 = 0; t2 < 2; ++t2)
#pragma unroll
                for (int s2 = 0; s2 < 2; ++s2) mma(acc[0], W0.get(FR_B3 + 2 * t2 + s2, lane), dH[t2][s2]);
            {
                Frag dh2;
                acc_to_frag<TM>(acc[0], 0, false, dh2);
                reinterpret_cast<h8v *>(a.tile_aux + slot * TILE_AUX + 128)[lane] = dh2;   // the Cin slot
            }
            if (FF && a.n_ff > 0) {   // dL/d frame features = sum over the tile of dCin rows 25.. (h0: acc 13..15)
                const float d0 = wave_sum(h == 0 ? acc[0][13] : 0.f);
                const float d1 = a.n_ff > 1 ? wave_sum(h == 0 ? acc[0][14] : 0.f) : 0.f;
                const float d2 = a.n_ff > 2 ? wave_sum(h == 0 ? acc[0][15] : 0.f) : 0.f;
                frame = __builtin_amdgcn_readfirstlane(frame);
                if (lane < a.n_ff) {
                    const float dv = lane == 0 ? d0 : (lane == 1 ? d1 : d2);
                    if (frame != ff_frame) {
                        if (ff_frame >= 0 && !ABL(512))   // ABL 512 (timing build): no frame-feature atomics
                            atomic_add_f32(a.grad_ff + (size_t)ff_frame * a.n_ff + lane, s_ff[lane]);
                        s_ff[lane] = dv;
                    } else {
                        s_ff[lane] += dv;
                    }
                }
                ff_frame = frame;
            }
            if (!a.no_dx) {   // dL/dSH -> view-direction part of dL/dtf[:3,:3] (run_network :1281)
                float g[9];
                float unused;
                half_sums(acc[0][8], g[0], g[4]);
                half_sums(acc[0][9], g[1], g[5]);
                half_sums(acc[0][10], g[2], g[6]);
                half_sums(acc[0][11], g[3], g[7]);
                half_sums(acc[0][12], g[8], unused);
                auto rdl = [&](float v, int l) {
                    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
                };
                const float vd[3] = {rdl(vdw.x, 0), rdl(vdw.y, 0), rdl(vdw.x, 1)};
                const float x = rdl(vdw.y, 1), y = rdl(vdw.x, 2), zz = rdl(vdw.y, 2);
                const float gdir[3] = {
                    -SH_C1 * g[3] + SH_C2_0 * y * g[4] + SH_C2_2 * (-2.f * x) * g[6] + SH_C2_3 * zz * g[7] +
                        SH_C2_4 * 2.f * x * g[8],
                    -SH_C1 * g[1] + SH_C2_0 * x * g[4] + SH_C2_1 * zz * g[5] + SH_C2_2 * (-2.f * y) * g[6] -
                        SH_C2_4 * 2.f * y * g[8],
                    SH_C1 * g[2] + SH_C2_1 * y * g[5] + SH_C2_2 * 4.f * zz * g[6] + SH_C2_3 * x * g[7]};
                const int i = (lane >> 2) % 3, j = lane & 3;
                const float gi = i == 0 ? gdir[0] : (i == 1 ? gdir[1] : gdir[2]);
                const float vj = j == 0 ? vd[0] : (j == 1 ? vd[1] : vd[2]);
                if (lane < 12 && j < 3) atomic_add_f32(a.ray_grad + (size_t)r * 12 + lane, gi * vj);
            }
            lds_wave_sync();
        } else {
            // L1 (X -> image 0, H1 -> images 1, 2)
            Frag X[2], H1[2][2];
            X[0] = in0;
            X[1] = in1;
#pragma unroll
            for (int mt = 0; mt < 2; ++mt) {
                acc_init_bias(acc[mt], s_b, mt, h);
#pragma unroll
                for (int s = 0; s < 2; ++s) mma(acc[mt], W1.get(FR_L1 + mt * 2 + s, lane), X[s]);
            }
            img_write(IMG(0), X, lane);
            advance();   // X (the prefetched operands) is consumed
            const float dsdf = sd.x * rw * lscale;
            if (h == 0) n_bwd += sd.z;
#pragma unroll
            for (int t = 0; t < 2; ++t)
#pragma unroll
                for (int s = 0; s < 2; ++s) acc_to_frag<TM>(acc[t], s, true, H1[t][s]);
            uint32_t r1[16];   // H1's ReLU factors, kept for dH1 below
            (void)relu_factors(H1, r1);
            img_write(IMG(1), H1[0], lane);
            img_write(IMG(2), H1[1], lane);
            // dH2: pass 0's sigma-net output gradient (colour tiles), the sdf loss gradient in row 0
            Frag dH2 = colour ? dh2in : zero;
            if (h == 0) frag_set<TM>(dH2, 0, dsdf);
            // dW2 += dH2^T H1, db2 (dH2 image: 3, units 0..15)
            img_write1(IMG(3), dH2, 0, lane);
            lds_wave_sync();
            dw16_tr(dwa[2], IMG(3), IMG(1), IMG(2), lane, &dba[2]);
            // dH1 = m1 (B2 dH2) (-> images 1, 2: H1 is done), dW1 += dH1^T X, db1
#pragma unroll
            for (int mt = 0; mt < 2; ++mt) {
                acc_zero(acc[mt]);
                mma(acc[mt], W1.get(FR_B2 + mt * 2, lane), dH2);
            }
            Frag dH1[2][2];
            masked_frags_r(acc, r1, dH1);
            lds_wave_sync();
            img_write(IMG(1), dH1[0], lane);
            img_write(IMG(2), dH1[1], lane);
            lds_wave_sync();
            dw_tr(dwa[0], IMG(1), IMG(0), lane, &dba[0]);
            dw_tr(dwa[1], IMG(2), IMG(0), lane, &dba[1]);
            lds_wave_sync();
            // dX = B1 dH1 -> feature gradients in this lane's level order
            acc_zero(acc[0]);
#pragma unroll
            for (int t2 = 0; t2 < 2; ++t2)
#pragma unroll
                for (int s2 = 0; s2 < 2; ++s2) mma(acc[0], W1.get(FR_B1 + 2 * t2 + s2, lane), dH1[t2][s2]);
            // (an out-of-box sample's column is exactly zero already: its dH2 is — every loss term and the
            // colour hand-off carry the sample-valid factor — and the MFMA columns are independent)
#pragma unroll
            for (int ss = 0; ss < 2; ++ss) {
                Frag f;
#pragma unroll
                for (int p = 0; p < 4; ++p) frag_put2(f, p, pk_round(acc[0][8 * ss + 2 * p], acc[0][8 * ss + 2 * p + 1]));
                store_dfeat<TM>(a.dfeat, (size_t)a.R * a.S, (size_t)sid0, n, ss, h, f);
            }
        }
    };
    // the first prefetch has landed before each loop (s_waitcnt vmcnt(0) as a builtin, which the
    // compiler's wait insertion tracks): entering a loop with it still counted, the loop header's
    // merged state would make every iteration wait on its own stores before the first MFMA
    __builtin_amdgcn_s_waitcnt(0x0f70);
    int li = li0;
    for (const int c_end = min(lend, n_c); li < c_end; li += lstep) tile(std::true_type{}, li);
    if constexpr (PASS == 1) {
        __builtin_amdgcn_s_waitcnt(0x0f70);
        for (; li < lend; li += lstep) tile(std::false_type{}, li);
        n_bwd = wave_sum(n_bwd);
        if (lane == 0) atomic_add_f32(loss_row(a, wg) + 5, n_bwd);
    }
    if constexpr (FF) {
        if (ff_frame >= 0 && lane < a.n_ff) atomic_add_f32(a.grad_ff + (size_t)ff_frame * a.n_ff + lane, s_ff[lane]);
    }
    dba[2] += __shfl_xor(dba[2], 16, 64);   // db5 / db2 (dw16_tr): lane groups 0 + 1, 2 + 3
    if constexpr (BLK) {   // the block's sums, one atomic per element (every wave takes part)
        amp_bwd_flush_block<PASS, NF, NB, PASS == 0 ? 3 : 2>(a, dwa, dba, smem, wave, lane, WPB);
        return;
    }
    if (li0 >= lend) return;   // no tiles: nothing to flush
    amp_bwd_flush<PASS, NF, NB>(a, dwa, dba, lane);
}
