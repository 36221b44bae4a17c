"""crimp_amd -- MI355X-native photon hot path of CRIMP (calcphase, Z^2/H periodicity search,
unbinned template-likelihood ToA scan) behind CRIMP's own Python API.

Drop-in modules keep the reference module names:
    crimp_amd.calcphase      calcphase, Phases
    crimp_amd.periodsearch   PeriodSearch (ztest, htest, twod_ztest, twod_htest)
    crimp_amd.templatemodels Fourier, WrappedCauchy, VonMises
    crimp_amd.measureToAs    measureToAs, measureToA_fourier/_cauchy/_vonmises, main (measuretoas CLI)
The hot loops run in libcrimp_hip.so (include/crimp_hip.h); see DESIGN.md.
"""
__version__ = "0.1.0"
