// search_mfma.h -- factorised (MFMA) periodicity search for arithmetic-progression trial grids.
// Returns 1 when it produced the result, 0 when it declines (caller falls back to the direct
// kernel), or a negative status on error.
static int mfma_search(Scratch& sc, hipStream_t s, const double* dt, const double* dt2, int64_t n,
                       const double* freq, int64_t nf, const double* c2, bool twod, int nharm, int stat,
                       int64_t first, int64_t count, double* out, uint32_t flags) {
    (void)sc; (void)s; (void)dt; (void)dt2; (void)n; (void)freq; (void)nf; (void)c2; (void)twod;
    (void)nharm; (void)stat; (void)first; (void)count; (void)out; (void)flags;
    return 0;
}
