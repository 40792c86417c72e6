/* hd_probe.h -- measured VALU issue rates used as roofline denominators
 * (bench.py).  op: 0 = v_add_u32, 1 = v_mad_u64_u32, 2 = v_mul_lo_u32,
 * 3 = v_mul_hi_u32 (+ v_add_u32).  ops_per_s counts lane-operations/s. */
#ifndef HD_PROBE_H
#define HD_PROBE_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif
int hd_probe_valu(int device, int op, uint32_t iters, double* ops_per_s);
#ifdef __cplusplus
}
#endif
#endif
