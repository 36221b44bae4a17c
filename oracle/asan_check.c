/*
 * asan_check.c -- AddressSanitizer / UBSan run of the CPU oracle (TEST INFRASTRUCTURE, `make -C oracle asan`).
 *
 * Compiles crimp_oracle.c into this driver with -fsanitize=address,undefined and calls every entry point on
 * small inputs, including the edge cases the tests use (one photon, one trial, empty glitch/wave lists, the
 * photon-blocked search branch, infeasible norms in the ToA grid). Exit status 0 and no sanitizer report is
 * the pass condition; the numbers themselves are checked by the Python tests against the golden vectors.
 */
#include "crimp_oracle.c"

#include <stdio.h>

static double urand(uint64_t* s) {
    *s = *s * 6364136223846793005ULL + 1442695040888963407ULL;
    return (double)(*s >> 11) * (1.0 / 9007199254740992.0);
}

int main(void) {
    uint64_t seed = 12345;
    /* calcphase: Taylor + glitch + wave terms, and a model with none of the optional parts */
    orc_model m;
    memset(&m, 0, sizeof(m));
    m.pepoch = 58000.0;
    m.f[0] = 0.1;
    m.f[1] = -1e-12;
    m.n_glitch = 2;
    for (int j = 0; j < 2; ++j) {
        m.glitch[j][0] = 58000.5 + j;
        m.glitch[j][1] = 0.1;
        m.glitch[j][2] = 1e-7;
        m.glitch[j][6] = j ? 10.0 : 0.0;
    }
    m.n_wave = 3;
    m.wave_epoch = 58000.0;
    m.wave_om = 0.01;
    for (int j = 0; j < 3; ++j) m.wave_ab[j][0] = m.wave_ab[j][1] = 1e-3;
    enum { NT = 1000 };
    double t[NT], tot[NT], fol[NT];
    for (int i = 0; i < NT; ++i) t[i] = 58000.0 + 3.0 * i / NT;
    orc_calcphase(t, NT, &m, 7, tot, fol);
    orc_calcphase(t, 1, &m, 1, tot, fol);
    m.n_glitch = 0;
    m.n_wave = 0;
    orc_calcphase(t, NT, &m, 7, tot, fol);

    /* searches: 1-D and 2-D grids, Z^2 and H, one photon, one trial, and the photon-blocked branch */
    enum { NP = 5000, NF = 37 };
    double *ts = malloc(sizeof(double) * (1 << 22)), f[NF], fd[3] = {-12.0, -10.0, -9.5}, out[3 * NF];
    for (int i = 0; i < NP; ++i) ts[i] = 5.0e9 + 1.0e4 * i / NP + 1e-3 * urand(&seed);
    for (int j = 0; j < NF; ++j) f[j] = 1.7 + (j - NF / 2) * 1e-5;
    const double t0 = (ts[0] + ts[NP - 1]) / 2;
    orc_search(ts, NP, t0, f, NF, NULL, 0, 2, 0, out);
    orc_search(ts, NP, t0, f, NF, fd, 3, 5, 1, out);
    orc_search(ts, 1, ts[0], f, 1, NULL, 0, 1, 0, out);
    const int64_t big = (int64_t)1 << 22;
    for (int64_t i = 0; i < big; ++i) ts[i] = 5.0e9 + 1.0e5 * (double)i / (double)big;
    orc_search(ts, big, (ts[0] + ts[big - 1]) / 2, f, 3, NULL, 0, 2, 0, out);
    free(ts);

    /* ToA likelihoods: Fourier, wrapped Cauchy, von Mises; the grid with infeasible low norms */
    enum { NX = 3000 };
    double x[NX], o[7];
    for (int i = 0; i < NX; ++i) x[i] = urand(&seed);
    const double p1[2] = {6.0, 3.0}, p2[2] = {1.0, 4.0}, p3[2] = {0.4, 0.9}, i0k[2] = {1.0, 1.0};
    double norms[20], phis[126], ll[20 * 126];
    for (int a = 0; a < 20; ++a) norms[a] = 0.05 + a * 25.0;
    for (int b = 0; b < 126; ++b) phis[b] = -ORC_PI + 0.05 * b;
    for (int model = 0; model < 3; ++model) {
        orc_toa_eval(x, NX, 250.0, model, 2, p1, p2, p3, i0k, 1.0, 5.0, 0.3, o);
        orc_toa_eval(x, 1, 250.0, model, 2, p1, p2, p3, i0k, 1.0, 0.01, 0.3, o);
        orc_toa_grid(x, NX, 250.0, model, 2, p1, p2, p3, i0k, 1.0, norms, 20, phis, 126, ll);
    }
    printf("asan_check: all oracle entry points ran clean\n");
    return 0;
}
