// mfma_drain.h -- keeping VALU writes and reads away from in-flight MFMAs on gfx950.
//
// Measured on the exact search kernel (two waves per SIMD mixing fp64 VALU work, LDS table reads and
// v_mfma_i32_32x32x32_i8): with hipcc's own scheduling, repeat runs and trial partitions differed by single
// photon terms (~1e-11..1e-9 relative) in result rows 16..31 of a tile, mostly in the second wave of each SIMD.
// Two code shapes were involved, and both are fixed here:
//   * operand overwrite: hipcc rewrote an MFMA's A registers (the next digit level's shifted operand) in the
//     very next instruction. Keeping the four level operands in distinct registers and issuing the quad's 8
//     MFMAs as a group (scheduling barriers) followed by mfma_operand_guard() -- 32 wait states, so the
//     earliest rewrite of an A register comes >= 48 issue cycles after its MFMA -- made every run
//     bit-identical; the same code without the group (A rewritten at once) stayed nondeterministic
//     (tools/dbg_part.py, tools/dbg_2d.py, tools/run_guard_ab.sh). Cost: ~2 % of the search.
//   * result read: hipcc pads 12 wait states between a 32x32 MFMA and a dependent VALU read, the edge of the
//     measured latency of the last result rows (tools/mb_hazard.hip: rows 0..15 land within ~8, rows 16..31
//     after ~12). mfma_drain() (256 wait states) precedes every read of the accumulators (once per fold).
// tools/mb_hazard.hip reproduces the result latency but not the operand hazard in isolation (single MFMAs,
// queued MFMAs, 4 waves per SIMD all read their operands in time), so the guard distances are empirical
// margins, enforced on the built code object by tools/isa_hazards.py (a CPU test).
#pragma once

// wait before VALU code reads MFMA results (this wave only; the other waves keep issuing)
__device__ __forceinline__ void mfma_drain() {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile(
        "s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7\n"
        "s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7\n"
        "s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7\n"
        "s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7");
    __builtin_amdgcn_sched_barrier(0);
}

// end of a group of MFMAs whose operands were all computed before the group: nothing may be scheduled into
// the group, and the next writes of the group's operand registers come after 32 wait states
__device__ __forceinline__ void mfma_operand_guard() {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7");
    __builtin_amdgcn_sched_barrier(0);
}
