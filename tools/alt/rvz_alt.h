/* rvz_alt.h — the leaf evaluator's A/B alternatives and parity cross-checks (tools/alt/librvz_alt.so).
 * NOT part of the product C-ABI (include/rvz.h): the product evaluator is rvz_resnet_fwd_h2.
 * These stay buildable so the tests can hold the h2 kernel against an exact-f32 MFMA forward and
 * so bench.py / tools can A/B them. Device pointers, stream-ordered, RVZ_* return codes. */
#ifndef RVZ_ALT_H
#define RVZ_ALT_H
#include "../../include/rvz.h"
#ifdef __cplusplus
extern "C" {
#endif

/* In place over an NHWC (channels_last) activation of n_pix pixels x channels (conv output with
 * the BN-folded conv bias not yet added): x = act(x + bias[c] (+ residual)), act = ReLU when
 * relu != 0 — network.py:23-28,97's bias/BN, skip add and ReLU in one pass after a MIOpen conv.
 * f32: channels % 4 == 0; bf16 (x, residual bf16, bias f32): channels % 8 == 0. */
int rvz_nn_bias_act_f32(float *x, const float *bias, const float *residual, int64_t n_pix,
                        int32_t channels, int32_t relu, void *hip_stream);
int rvz_nn_bias_act_bf16(void *x, const float *bias, const void *residual, int64_t n_pix,
                         int32_t channels, int32_t relu, void *hip_stream);

/* The whole forward on the f32-input MFMA (board 8; exact k-ordered fp32 FMA chains). params:
 * rvz.network.pack_resnet_params (rvz_resnet_params_size floats, 16-byte aligned). */
int rvz_resnet_fwd_f32(int32_t board, const float *x, int32_t n, const float *params,
                       int32_t filters, int32_t blocks, float *logits, float *value,
                       void *hip_stream);

/* fp32 as a 3-part bf16 split, six partial products (boards 8 and 6): wsplit from
 * rvz_resnet_split_weights (rvz_resnet_split_size uint16), work rvz_resnet_work_size(n) floats. */
int64_t rvz_resnet_split_size(int32_t filters, int32_t blocks);
int rvz_resnet_split_weights(const float *params, int32_t filters, int32_t blocks,
                             uint16_t *wsplit, void *hip_stream);
int rvz_resnet_fwd_split(int32_t board, const float *x, int32_t n, const float *params,
                         const uint16_t *wsplit, int32_t filters, int32_t blocks, float *work,
                         float *logits, float *value, void *hip_stream);
int rvz_resnet_trunk_split(int32_t board, const float *x, int32_t n, const float *params,
                           const uint16_t *wsplit, int32_t filters, int32_t blocks, float *work,
                           void *hip_stream);
/* The FC heads (work -> logits, value) on the VALU: k_heads_mfma's predecessor. */
int rvz_alt_heads_valu(int32_t board, const float *work, int32_t n, const float *params,
                       int32_t filters, int32_t blocks, float *logits, float *value,
                       void *hip_stream);

/* out[i] = the engine's sqrt_count(i) (csrc/rvz_engine.hip) for i < n, same compile flags. */
int rvz_alt_sqrt_count(int32_t n, float *out, void *hip_stream);
/* out[i] = x[i] ** e[i] in float64: mode 1 = k_act's correctly rounded power (csrc/rvz_pow.hip.h),
 * mode 0 = the device library's pow; rvz_alt_pow_host = the same pow_cr compiled for the host. */
int rvz_alt_pow(int32_t n, const double *x, const double *e, double *out, int32_t mode,
                void *hip_stream);
int rvz_alt_pow_host(int32_t n, const double *x, const double *e, double *out);

#ifdef __cplusplus
}
#endif
#endif /* RVZ_ALT_H */
