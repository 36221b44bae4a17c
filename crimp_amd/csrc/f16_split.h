// f16_split.h -- fp32 -> (hi, lo) f16 pairs for exact fp32 products on the f16 matrix cores (k_toa_grid_mf).
// hi = RN_f16(x), lo = RN_f16(x - hi): |x - hi - lo| <= 2^-22 |x|, so hi.hi + hi.lo + lo.hi + lo.lo of two split
// operands carry an fp32 product.
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Two values at once: hi = (RN(x), RN(y)) in one conversion, lo = (RN(x - hi.x), RN(y - hi.y)); NEGY splits -y.
// Explicit instructions: left alone, the compiler may fuse a producing multiply into one conversion but not the
// other, so that hi + lo != x (that bug gave 1e-5 errors on squared harmonics).
template <bool NEGY>
__device__ __forceinline__ void split_xy(float x, float y, uint32_t& dh, uint32_t& dl) {
    if (NEGY)
        asm volatile(
            "v_cvt_pk_f16_f32 %0, %2, -%3\n\t"
            "v_fma_mixlo_f16 %1, %2, 1.0, -%0 op_sel_hi:[0,0,1]\n\t"
            "v_fma_mixhi_f16 %1, -%3, 1.0, -%0 op_sel:[0,0,1] op_sel_hi:[0,0,1]"
            : "=&v"(dh), "=&v"(dl)
            : "v"(x), "v"(y));
    else
        asm volatile(
            "v_cvt_pk_f16_f32 %0, %2, %3\n\t"
            "v_fma_mixlo_f16 %1, %2, 1.0, -%0 op_sel_hi:[0,0,1]\n\t"
            "v_fma_mixhi_f16 %1, %3, 1.0, -%0 op_sel:[0,0,1] op_sel_hi:[0,0,1]"
            : "=&v"(dh), "=&v"(dl)
            : "v"(x), "v"(y));
}
