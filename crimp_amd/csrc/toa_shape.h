// Extended-LL sums with template-shape gradients (crimp_toa_shape_points), for ToA fits that free
// template parameters (readvaryparam, measureToAs.py:727-801). Included by crimp_hip.hip.
//
// One 256-thread block per point (interval + its own template + norm + phShift); threads stride
// the interval's photons. Per photon and component j (x in cycles for Fourier, radians otherwise):
//   fourier   u = 2 pi (j+1) x + ph_j - (j+1) phi,  h_j = A a_j cos u
//             dh/da_j = A cos u, dh/dph_j = -A a_j sin u, dh/dphi = (j+1) A a_j sin u
//   cauchy    v = x - cen_j - phi, D = cosh w - cos v, h_j = (A a_j / 2 pi) sinh w / D
//             dh/da_j = h_j / a_j, dh/dcen_j = dh/dphi = (A a_j / 2 pi) sinh w sin v / D^2,
//             dh/dw_j = (A a_j / 2 pi) (1 - cosh w cos v) / D^2
//   vonmises  k = 1/w^2, e = exp(k cos v) / (2 pi I0(k)), h_j = A a_j e
//             dh/da_j = A e, dh/dcen_j = dh/dphi = A a_j e k sin v,
//             dh/dw_j = A a_j e (cos v - I1(k)/I0(k)) (-2 / w^3)
// (templatemodels.py:64-82, 166-185, 271-290 differentiated). fp64 throughout.

constexpr int kShapeBlock = 256;
constexpr int kShapeSums = CRIMP_SHAPE_SUMS;

struct ShapeComp {  // per component, derived once per block
    double a;       // A a_j (fourier), A a_j / 2 pi (cauchy), A a_j / (2 pi I0) (vonmises)
    double A;       // dh/da_j factor: A (fourier), A / 2 pi (cauchy), A / (2 pi I0) (vonmises)
    double c, s;    // cos/sin(ph_j - (j+1) phi) (fourier) or cos/sin(cen_j + phi)
    double ch, sh;  // cosh w, sinh w (cauchy)
    double k, r, w; // 1/w^2, I1/I0, w (vonmises)
};

template <int MODEL>
__global__ __launch_bounds__(kShapeBlock) void k_toa_shape(const double* __restrict__ x,
                                                           const int64_t* __restrict__ offsets,
                                                           const crimp_template* __restrict__ tpls,
                                                           const double* __restrict__ aux,
                                                           const int64_t* __restrict__ pt_interval,
                                                           const double* __restrict__ pt_norm,
                                                           const double* __restrict__ pt_phi,
                                                           double* __restrict__ out) {
    __shared__ ShapeComp comp[CRIMP_MAX_COMP];
    __shared__ double red[kShapeBlock / 64][kShapeSums];
    __shared__ double gacc[3 * CRIMP_MAX_COMP][kShapeBlock];  // per-thread gradient sums (98 KB LDS)
    const int64_t p = blockIdx.x;
    const int tid = threadIdx.x;
    const crimp_template* tp = tpls + p;
    constexpr int model = MODEL;
    const int K = tp->ncomp;
    const double phi = pt_phi[p], nrm = pt_norm[p];
    const double twopi = 6.283185307179586476925286766559;
    if (tid < K) {
        const int j = tid;
        ShapeComp q{};
        const double A = tp->amp_shift;
        if (model == CRIMP_MODEL_FOURIER) {
            q.A = A;
            q.a = A * tp->amp[j];
            sincos(tp->loc[j] - (double)(j + 1) * phi, &q.s, &q.c);
        } else {
            sincos(tp->loc[j] + phi, &q.s, &q.c);
            q.w = tp->wid[j];
            if (model == CRIMP_MODEL_CAUCHY) {
                q.A = A / twopi;
                q.ch = cosh(q.w);
                q.sh = sinh(q.w);
            } else {
                q.A = A / (twopi * tp->i0[j]);
                q.k = 1.0 / (q.w * q.w);
                q.r = aux != nullptr ? aux[p * CRIMP_MAX_COMP + j] : 0.0;
            }
            q.a = q.A * tp->amp[j];
        }
        comp[j] = q;
    }
    __syncthreads();

    double acc[4] = {0.0, INFINITY, 0.0, 0.0};
    for (int q = 0; q < 3 * CRIMP_MAX_COMP; ++q) gacc[q][tid] = 0.0;
    const int64_t iv = pt_interval[p];
    const int64_t a0 = offsets[iv], b0 = offsets[iv + 1];
    // two passes over the components per photon: the model m first, then the gradient terms / m
    // (the 3K gradient sums live in LDS, one column per thread: conflict-free, no register spills)
    for (int64_t i = a0 + tid; i < b0; i += kShapeBlock) {
        double s1, c1;
        photon_sincos(model, x[i], s1, c1);
        double h = 0.0, hphi = 0.0;
        double cj = c1, sj = s1;  // fourier: cos/sin(2 pi (j+1) x) by recurrence
        for (int j = 0; j < K; ++j) {
            const ShapeComp& q = comp[j];
            if (model == CRIMP_MODEL_FOURIER) {
                const double cu = cj * q.c - sj * q.s, su = sj * q.c + cj * q.s;
                h += q.a * cu;
                hphi += (double)(j + 1) * q.a * su;
                const double cn = cj * c1 - sj * s1;
                sj = sj * c1 + cj * s1;
                cj = cn;
            } else {
                const double cv = c1 * q.c + s1 * q.s;  // cos(x - cen - phi)
                const double sv = s1 * q.c - c1 * q.s;  // sin(x - cen - phi)
                if (model == CRIMP_MODEL_CAUCHY) {
                    const double iD = 1.0 / (q.ch - cv);
                    h += q.a * q.sh * iD;
                    hphi += q.a * q.sh * sv * iD * iD;
                } else {
                    const double v = q.a * exp(q.k * cv);
                    h += v;
                    hphi += v * q.k * sv;
                }
            }
        }
        const double mv = nrm + h;
        const double iq = 1.0 / mv;
        acc[0] += log(mv);
        acc[1] = fmin(acc[1], mv);
        acc[2] += iq;
        acc[3] += hphi * iq;
        cj = c1;
        sj = s1;
        for (int j = 0; j < K; ++j) {
            const ShapeComp& q = comp[j];
            if (model == CRIMP_MODEL_FOURIER) {
                const double cu = cj * q.c - sj * q.s, su = sj * q.c + cj * q.s;
                gacc[3 * j][tid] += q.A * cu * iq;
                gacc[3 * j + 1][tid] -= q.a * su * iq;
                const double cn = cj * c1 - sj * s1;
                sj = sj * c1 + cj * s1;
                cj = cn;
            } else {
                const double cv = c1 * q.c + s1 * q.s;
                const double sv = s1 * q.c - c1 * q.s;
                if (model == CRIMP_MODEL_CAUCHY) {
                    const double iD = 1.0 / (q.ch - cv);
                    const double iD2 = iD * iD * iq;
                    gacc[3 * j][tid] += q.A * q.sh * iD * iq;
                    gacc[3 * j + 1][tid] += q.a * q.sh * sv * iD2;
                    gacc[3 * j + 2][tid] += q.a * (1.0 - q.ch * cv) * iD2;
                } else {
                    const double e = exp(q.k * cv) * iq;
                    gacc[3 * j][tid] += q.A * e;
                    gacc[3 * j + 1][tid] += q.a * e * q.k * sv;
                    gacc[3 * j + 2][tid] += q.a * e * (cv - q.r) * (-2.0 / (q.w * q.w * q.w));
                }
            }
        }
    }
    const int wid = tid >> 6, lane = tid & 63;
    for (int q = 0; q < kShapeSums; ++q) {
        const double a = q < 4 ? acc[q] : gacc[q - 4][tid];
        const double v = q == 1 ? wave_min(a) : wave_sum(a);
        if (lane == 0) red[wid][q] = v;
    }
    __syncthreads();
    if (tid < kShapeSums) {
        double v = red[0][tid];
        for (int w = 1; w < kShapeBlock / 64; ++w) v = tid == 1 ? fmin(v, red[w][tid]) : v + red[w][tid];
        out[p * kShapeSums + tid] = v;
    }
}
