/* Lab C-ABI of the persistent decode engine (tools/lab/engine/engine.hip): measured slower than the product's
 * per-op decode graph, so it lives outside liblitgpt_amd.so, in
 * tools/_lab/liblga_engine.so (make -C lit-gpt_amd/csrc lab-engine), which also carries the product objects. */
#ifndef LGA_ENGINE_LAB_H
#define LGA_ENGINE_LAB_H
#include "litgpt_amd.h"
#ifdef __cplusplus
extern "C" {
#endif

/* -- persistent decode engine: the WHOLE greedy decode step in one launch ---------------------------------
 * Replaces, for one token of generate/base.py's decode loop (next_token -> GPT.forward -> 32 x Block.forward ->
 * ln_f -> lm_head -> sample at temperature 0; generate/base.py:44-47,87-92, lit_gpt/model.py:499-519,572-593,
 * 609-656,712-716), the 160-launch chain of the kernels above. One workgroup per CU: a loader wave streams every
 * weight row and K/V row the CU owns into an LDS ring with LDS-DMA, running ahead across op boundaries, while
 * consumer waves compute (RMSNorm + int4 GEMV with the same arithmetic as lga_q4_gemv / lga_q4_gemv_swiglu,
 * RoPE + KV append + split attention, argmax + next embedding) and hand activations between CUs through
 * write-through stores and per-op arrival counters.
 * Llama-family blocks only (RMSNorm, LLaMAMLP, no bias, head_size == rope_n_elem == 128), 4-bit weights of one
 * format, tensor-parallel world 1; lga_engine_check says whether a geometry is covered.
 * layers: DEVICE array of n_layer lga_engine_layer. x0: the step's input embedding (n_embd bf16) lives in the
 * scratch (lga_engine_x0); the launch writes the next token's embedding there, the token into *token,
 * *pos += 1, and out_idx (if not NULL) <- token. logits (vocab bf16, may be NULL) receives the step's logits.
 * scratch: lga_engine_scratch_bytes(g) bytes, zeroed before the first launch (and by lga_engine_reset after an
 * error); err (lga_engine_error) is non-zero after a launch that gave up waiting (results invalid).
 * op_limit > 0 stops after that many ops (test hook: 5 ops per block, the lm_head + argmax last). */
typedef struct lga_engine_layer {
  const void* qkv_w;   /* (H + 2G) hs x C/2 packed nibbles; qkv_s its scales */
  const void* qkv_s;
  const void* o_w;     /* attn.proj C x C/2 */
  const void* o_s;
  const void* fc1_w;   /* mlp.fc_1 I x C/2 */
  const void* fc1_s;
  const void* fc2_w;   /* mlp.fc_2 I x C/2 */
  const void* fc2_s;
  const void* dn_w;    /* mlp.proj C x I/2 */
  const void* dn_s;
  const void* norm1;   /* norm_1.weight (C bf16) */
  const void* norm2;   /* norm_2.weight */
  void* k_cache;       /* (G, max_seq, hs) bf16 */
  void* v_cache;
} lga_engine_layer;

typedef struct lga_engine_geom {
  int n_layer, n_embd, n_head, n_query_groups, head_size, intermediate, vocab, max_seq;
  int group, fmt, rope_rows, n_cu;
  float norm_eps, attn_scale;
} lga_engine_geom;

int lga_engine_check(const lga_engine_geom* g);
size_t lga_engine_scratch_bytes(const lga_engine_geom* g);
void* lga_engine_x0(const lga_engine_geom* g, void* scratch);
int lga_engine_reset(const lga_engine_geom* g, void* scratch, lga_stream_t stream);
int lga_engine_error(const lga_engine_geom* g, const void* scratch, unsigned* err_out);
int lga_decode_engine(const lga_engine_geom* g, const lga_engine_layer* layers, const void* lm_w, const void* lm_s,
                      const void* ln_f, const void* wte, const float* cos, const float* sin, int64_t* pos,
                      int32_t* token, int64_t* out_idx, void* logits, void* scratch, int op_limit,
                      lga_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* LGA_ENGINE_LAB_H */
