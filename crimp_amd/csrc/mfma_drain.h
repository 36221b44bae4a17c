// mfma_drain.h -- wait for the matrix pipe before VALU code reads MFMA results (gfx950).
//
// hipcc pads 12 wait states between a v_mfma_*_32x32x* and a dependent VALU read. tools/mb_hazard.hip measures
// the result latency of v_mfma_i32_32x32x32_i8: rows 0..15 land within ~8 wait states, rows 16..31 (result
// registers 8..15) after ~12, i.e. at the padding's edge. In the search kernels, with two waves per SIMD
// mixing fp64 VALU work and MFMAs, reads placed 40+ issue cycles after the last MFMA by the compiler still
// saw stale partial sums in rows 16..31 now and then: rare, timing-dependent errors of single photon terms
// in rows a >= 16 of a tile (repeat runs and trial partitions differed). The kernels therefore drain before
// every read of their accumulators: 256 wait states (this wave only; the other waves keep issuing), placed
// where the accumulators are read once per fold or chunk, and fenced against scheduling across it.
// tools/isa_hazards.py checks the built code object for result reads that come too early.
#pragma once

__device__ __forceinline__ void mfma_drain() {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile(
        "s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7\n"
        "s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7\n"
        "s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7\n"
        "s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7");
    __builtin_amdgcn_sched_barrier(0);
}
