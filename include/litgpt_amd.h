/*
 * litgpt_amd.h — C ABI of liblitgpt_amd.so, the MI355X (gfx950) hot path of lit_gpt's quantized decode.
 *
 * Conventions: plain device pointers + sizes, no torch types; every buffer is caller-owned
 * (kernels never allocate; scratch is passed in); all launches are asynchronous on `stream` (a hipStream_t;
 * graph-capturable); return 0 on success, otherwise a hipError_t value with a message available from
 * lga_last_error_string() (thread-local). bf16 tensors are raw uint16 bit patterns, row-major, contiguous.
 *
 * Reference interfaces replaced (file:line in /root/reference unless marked upstream):
 *   - bitsandbytes 0.41.0 (requirements-all.txt:3; upstream, not in the reference tree) reached via Lightning's
 *     BitsandbytesPrecision (generate/base.py:128-136, generate/tp.py:126-134,171,190): the ctypes C functions
 *     cquantize_blockwise_bf16_nf4 / cdequantize_blockwise_bf16_nf4 / cgemm_4bit_inference_naive_bf16
 *     (upstream names) behind Linear4bit.forward -> lga_quantize, lga_q4_gemv(_swiglu), lga_q4_gemm;
 *   - the ATen kernels lit_gpt/model.py issues on the hot path -> the remaining entry points.
 */
#ifndef LITGPT_AMD_H
#define LITGPT_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ihipStream_t* lga_stream_t; /* == hipStream_t */

/* weight formats */
#define LGA_FMT_Q4G 0 /* int4, symmetric, per-group bf16 scale = bf16(absmax/7), nibble = q + 8 */
#define LGA_FMT_NF4 1 /* bitsandbytes NF4 codebook, per-block fp32 absmax */
#define LGA_FMT_BF16 2 /* unquantized bf16 weight [N][K] (lga_q4_gemm_fused / lga_q4_gemm_swiglu only) */
#define LGA_FMT_FP4 3 /* bitsandbytes FP4 code (get_4bit_type('fp4'), "bnb.fp4"), per-block fp32 absmax */

/* -- plumbing ---------------------------------------------------------------------------------------- */
const char* lga_last_error_string(void);
int lga_version(void);
int lga_device_info(int device, int* n_cu, char* arch_name, int arch_len);
/* builds the device objects of the prefill path's kernels (fused GEMM, flash attention, norms, RoPE, embedding,
 * lm_head GEMV, argmax) now instead of at their first launch, where the runtime spends about 0.5 ms per kernel
 * inside the first prompt (called by build_model, the model-load step; nothing is launched) */
int lga_preload_kernels(void);

/* -- quantize at load (Lightning BitsandbytesPrecision.convert_module + bnb quantize on .to(device);
 *    generate/base.py:168, generate/tp.py:171-190) ------------------------------------------------------
 * w: (N, K) fp32 (w_is_bf16 = 0) or bf16 (1). qweight: (N, K/2) bytes, byte j = k 2j (low) | 2j+1 (high).
 * scales: (N, K/group) bf16 for Q4G, fp32 for NF4 / FP4. Layout spec: oracle/quant.py. Every 4-bit entry point
 * below takes fmt 0 / 1 / 3 (FP4 runs the NF4 kernels with its own 16-entry codebook). */
int lga_quantize(const void* w, int w_is_bf16, uint8_t* qweight, void* scales, int N, int K, int group, int fmt,
                 lga_stream_t stream);
/* bitsandbytes double quantization of nf4 / fp4 statistics ("bnb.nf4-dq", "bnb.fp4-dq"; quantize_4bit(compress_statistics=True),
 * generate/base.py:105): absmax (n fp32, bnb's flattened 64-blocks, i.e. the NF4 scales of lga_quantize) is
 * replaced in place by code[q] * absmax2 + offset — q = nearest entry of `code` (the 256-entry signed dynamic
 * map, device fp32) to (absmax - offset) / absmax2 per block of 256, offset = mean(absmax) (written to
 * offset_out) — the statistic bnb's dequantize_4bit reconstructs. */
int lga_nf4_double_quant(float* absmax, long n, const float* code, float* offset_out, lga_stream_t stream);

/* -- decode GEMV, M = 1 (bnb gemv_4bit for one-token inputs; every Linear of lit_gpt/model.py:519,619,656,
 *    712-716) -----------------------------------------------------------------------------------------------
 * y[N] = x[K] . dequant(W)^T (+bias[N]) (+residual[N]); norm_weight != NULL applies RMSNorm
 * (lit_gpt/rmsnorm.py:19-25, eps = norm_eps) to x first. variant < 0 = heuristic tile choice. */
int lga_q4_gemv(const void* x, const uint8_t* qweight, const void* scales, const void* bias, const void* residual,
                const void* norm_weight, float norm_eps, void* y, int N, int K, int group, int fmt, int variant,
                lga_stream_t stream);
/* y[N] = bf16(silu(bf16(x.W1^T))) * bf16(x.W2^T) — LLaMAMLP fc_1/fc_2 + silu*mul (lit_gpt/model.py:712-715) */
int lga_q4_gemv_swiglu(const void* x, const uint8_t* qweight1, const void* scales1, const uint8_t* qweight2,
                       const void* scales2, const void* norm_weight, float norm_eps, void* y, int N, int K,
                       int group, int fmt, int variant, lga_stream_t stream);

/* -- prefill GEMM, M > 1 (bnb dequantize_4bit + cuBLAS GEMM) -------------------------------------------- */
int lga_q4_gemm(const void* x, const uint8_t* qweight, const void* scales, const void* bias, const void* residual,
                void* y, int M, int N, int K, int group, int fmt, lga_stream_t stream);
/* The same product with the dequantization fused into a 256 x 128 MFMA tile (csrc/gemm_q4f.hip): the weight
 * is never written out in bf16. fmt 0 int4-g / 1 nf4 / 2 bf16 weights [N][K] / 3 fp4; needs N % 8 == 0, K % 64 == 0 and
 * (4-bit) a power-of-two group >= 64 dividing K (lga_q4f_fits). Numerically the bnb path: bf16(value * scale)
 * weights, fp32 accumulation, one bf16 rounding (+bias), then + residual. */
int lga_q4f_fits(int M, int N, int K, int group, int fmt);
/* Short prompts split K across workgroups: the caller passes a zero-initialised workspace of at least this many
 * bytes (0 = none needed) and keeps it for later calls (its per-tile counters are left zeroed). */
size_t lga_q4f_workspace_bytes(int M, int N, int K, int swiglu);
int lga_q4_gemm_fused(const void* x, const void* weight, const void* scales, const void* bias, const void* residual,
                      void* y, int M, int N, int K, int group, int fmt, void* workspace, size_t workspace_bytes,
                      lga_stream_t stream);
/* LLaMAMLP prefill (lit_gpt/model.py:712-716): y (M, N) = bf16(silu(bf16(x W1^T))) * bf16(x W2^T), fc_1 and fc_2
 * in one launch (each tile computes 64 columns of both and applies the product in its epilogue). */
int lga_q4_gemm_swiglu(const void* x, const void* qweight1, const void* scales1, const void* qweight2,
                       const void* scales2, void* y, int M, int N, int K, int group, int fmt, void* workspace,
                       size_t workspace_bytes, lga_stream_t stream);
/* bnb dequantize_4bit (the first half of the reference's M > 1 Linear4bit path): w (N, K) bf16 =
 * bf16(value(nibble) * scale) — the same bits lga_q4_gemm / lga_q4_gemm_fused stage, so lga_bf16_gemm over w ==
 * lga_q4_gemm (tests, tools). */
int lga_q4_dequantize(const uint8_t* qweight, const void* scales, void* w, int N, int K, int group, int fmt,
                      lga_stream_t stream);

/* -- unquantized bf16 Linears (BASELINE config 2: no --quantize, precision bf16-true; the reference runs
 *    F.linear on the bf16 nn.Linear weight, lit_gpt/model.py:619, :656, :712-716, :519) ------------------- */
/* decode GEMV y (N) = x (K) . W (N, K)^T [+bias] [+residual]; optional fused RMSNorm of x (as lga_q4_gemv) */
int lga_bf16_gemv(const void* x, const void* weight, const void* bias, const void* residual, const void* norm_weight,
                  float norm_eps, void* y, int N, int K, lga_stream_t stream);
/* y = bf16(silu(bf16(x W1^T))) * bf16(x W2^T) (LLaMAMLP, model.py:715), optional fused RMSNorm of x */
int lga_bf16_gemv_swiglu(const void* x, const void* weight1, const void* weight2, const void* norm_weight,
                         float norm_eps, void* y, int N, int K, lga_stream_t stream);
/* prefill GEMM Y (M, N) = X (M, K) . W (N, K)^T [+bias] [+residual] on MFMA; K % 32 == 0 */
int lga_bf16_gemm(const void* x, const void* weight, const void* bias, const void* residual, void* y, int M, int N,
                  int K, lga_stream_t stream);

/* -- row / elementwise ops ---------------------------------------------------------------------------- */
/* RMSNorm over rows of n (lit_gpt/rmsnorm.py:19-25) */
int lga_rmsnorm(const void* x, const void* weight, void* y, int rows, int n, float eps, lga_stream_t stream);
/* RoPE (lit_gpt/model.py:641-644, 767-773) on the q and k slots of qkv (T, (H+2G)*hs) [per group g: q_per_kv
 * q heads, k, v — scripts/convert_hf_checkpoint.py:174-188 layout], cos/sin rows rope_pos[t] of (rope_rows,
 * rope_n_elem) fp32 tables; q_out (T, H, hs); k (roped) and v written to k_cache/v_cache (G, max_seq, hs) at row
 * cache_pos[t] (KVCache.forward index_copy_, lit_gpt/model.py:788-795). */
int lga_rope_kv_append(const void* qkv, void* q_out, void* k_cache, void* v_cache, const int64_t* cache_pos,
                       const int64_t* rope_pos, const float* cos, const float* sin, int rope_rows, int T, int n_head,
                       int n_query_groups, int head_size, int rope_n_elem, int max_seq, lga_stream_t stream);
/* out[t] = table[idx[t]] (nn.Embedding, lit_gpt/model.py:515) */
int lga_embedding(const void* idx, int idx_is_int64, const void* table, void* out, int T, int C, int V,
                  lga_stream_t stream);
/* y = bf16(a + b) (Block residual, lit_gpt/model.py:591-592) */
int lga_add(const void* a, const void* b, void* y, long n, lga_stream_t stream);
/* y = bf16(bf16(silu(a)) * b) (lit_gpt/model.py:715) */
int lga_swiglu(const void* a, const void* b, void* y, long n, lga_stream_t stream);
/* torch.nn.LayerNorm over rows of n (GPT-NeoX norm_class, lit_gpt/config.py:137-144; model.py:578-588):
 * fp32 mean / biased variance, y = bf16((x - mean) * rstd * weight + bias); bias may be NULL */
int lga_layernorm(const void* x, const void* weight, const void* bias, void* y, int rows, int n, float eps,
                  lga_stream_t stream);
/* y = bf16(gelu(a)) — GptNeoxMLP (lit_gpt/model.py:699-702): exact erf form, or tanh form when approximate_tanh */
int lga_gelu(const void* a, void* y, long n, int approximate_tanh, lga_stream_t stream);

/* -- attention over the KV cache (SDPA with the input_pos mask rows, lit_gpt/model.py:651,658-665) --------
 * q (T, H, hs); caches (G, max_seq, hs); query t attends keys 0..input_pos[t]; y (T, H*hs).
 * n_splits > 1 splits keys 0..input_pos[t] evenly (flash-decoding; the split merge happens in the same launch
 * by the last-arriving workgroup) and needs `workspace` of lga_attention_workspace_bytes(T, H, hs, n_splits) bytes
 * plus `counters` (T * H * 64 uint32 — one per (t, group, head slice) at a 256-B stride so the device-scope
 * atomics do not share a line; zeroed once at allocation, re-armed by the kernel; at T = 1 a group's heads may be
 * dealt to up to H/G workgroups when the groups are few).
 * head_size in {64, 128}; H/G in {1,2,4,8}; 1 <= n_splits <= 256. */
int lga_attention(const void* q, const void* k_cache, const void* v_cache, const int64_t* input_pos, void* y,
                  float* workspace, unsigned* counters, int T, int n_head, int n_query_groups, int head_size,
                  int max_seq, int n_splits, float scale, lga_stream_t stream);
size_t lga_attention_workspace_bytes(int T, int n_head, int head_size, int n_splits);
/* Decode step (T = 1) with RoPE + KV-append fused into the attention launch (apply_rope lit_gpt/model.py:641-644,
 * KVCache.forward :788-795, SDPA :651): qkv is the fused projection row ([G][q_per_kv + 2][hs], the layout of
 * CausalSelfAttention.attn); q and k are roped with row rope_pos[0] of cos/sin (rope_rows x 128 fp32); k, v are
 * stored at cache_pos[0]; y (H*hs) = attention of the roped q over keys 0..cache_pos[0]. Caches bit-identical to
 * lga_rope_kv_append; y equals lga_attention's up to fp32 summation order (the new key is scored last).
 * Requires head_size == rope_n_elem == 128. */
int lga_attention_decode_fused(const void* qkv, void* k_cache, void* v_cache, const int64_t* cache_pos,
                               const int64_t* rope_pos, const float* cos, const float* sin, int rope_rows, void* y,
                               float* workspace, unsigned* counters, int n_head, int n_query_groups, int head_size,
                               int rope_n_elem, int max_seq, int n_splits, float scale, lga_stream_t stream);

/* -- sparse MoE (LLaMAMoE.forward, lit_gpt/model.py:727-743; Mixtral) ------------------------------------------
 * lga_moe_route: per token row of router logits [T][n_expert] bf16 -> expert_ids [T][k] int32 and probs [T][k]
 * bf16 = topk(router, k) with the CPU torch.topk order on ties (model.py:737) and
 * softmax(dim=1, dtype=float).to(bf16) (model.py:738). n_expert <= 8. */
int lga_moe_route(const void* logits, int T, int n_expert, int k, int32_t* expert_ids, void* probs,
                  lga_stream_t stream);
/* lga_moe_gate_route: one token's router gate (the 4-bit `self.gate(x)` Linear, model.py:736, optional fused
 * RMSNorm of x as lga_q4_gemv) and its routing (lga_moe_route) in one launch: expert_ids [k] int32, probs [k] bf16,
 * bit-identical to lga_q4_gemv (n_expert rows) followed by lga_moe_route. n_expert <= 8, K <= 6144. */
int lga_moe_gate_route(const void* x, const uint8_t* qweight, const void* scales, const void* norm_weight,
                       float norm_eps, int n_expert, int K, int group, int fmt, int k, int32_t* expert_ids, void* probs,
                       lga_stream_t stream);
/* Routed expert GEMVs (the per-expert `expert(x[token_idx])` calls, model.py:741-742, for one token): slot s
 * (0..n_slots-1) uses expert e = expert_ids[s], whose packed weights / scales start at qweight + e * w_stride
 * bytes / scales + e * s_stride bytes (experts stacked with a uniform stride). lga_q4_gemv_experts reads
 * x + s * x_stride and writes y[s][N]; the SwiGLU form (fc_1 / fc_2 of LLaMAMLP, model.py:712-715) shares x and
 * optionally fuses RMSNorm (norm_2) like lga_q4_gemv_swiglu. */
int lga_q4_gemv_experts(const void* x, const uint8_t* qweight, const void* scales, const int32_t* expert_ids,
                        int n_slots, int n_expert, long long w_stride, long long s_stride, int x_stride, void* y,
                        int N, int K, int group, int fmt, int variant, lga_stream_t stream);
int lga_q4_gemv_swiglu_experts(const void* x, const uint8_t* qweight1, const void* scales1, const uint8_t* qweight2,
                               const void* scales2, const int32_t* expert_ids, int n_slots, int n_expert,
                               long long w_stride, long long s_stride, const void* norm_weight, float norm_eps,
                               void* y, int N, int K, int group, int fmt, int variant, lga_stream_t stream);
/* lga_q4_gemv_experts_pair_combine: one token, k = 2, no tensor parallelism — the routed proj GEMVs of both slots
 * (x [2][K] = the slots' SwiGLU rows, experts stacked as lga_q4_gemv_experts, expert_ids [2], probs [2]) and
 * lga_moe_combine with the Block residual in one launch: y [N] = residual + sum in ascending expert id of
 * bf16(probs[s] * expert_out[s]), bit-identical to lga_q4_gemv_experts + lga_moe_combine. The second-arriving
 * workgroup of each row block combines: `scratch` [2][N] bf16 holds the first one's rows (write-through),
 * `counters` (lga_q4_gemv_experts_pair_counters(N) words, caller-zeroed once) are re-armed by the kernel. */
int lga_q4_gemv_experts_pair_supported(int N, int K, int group, int fmt);
size_t lga_q4_gemv_experts_pair_counters(int N);
int lga_q4_gemv_experts_pair_combine(const void* x, const uint8_t* qweight, const void* scales,
                                     const int32_t* expert_ids, const void* probs, const void* residual, int n_expert,
                                     long long w_stride, long long s_stride, void* y, void* scratch,
                                     unsigned* counters, int N, int K, int group, int fmt, lga_stream_t stream);
/* y[t] = residual[t] (optional) + the bf16 sum, in ascending expert order, of bf16(probs[t][s] * expert_out[t][s])
 * (the `y[token_idx] += probs * expert(...)` loop, model.py:739-742, then Block's residual add model.py:592). */
int lga_moe_combine(const void* expert_out, const void* probs, const int32_t* expert_ids, const void* residual,
                    void* y, int T, int k, int C, lga_stream_t stream);
/* Grouped sparse-MoE prefill (T > 1): replaces the per-expert loop of LLaMAMoE.forward (model.py:740-742:
 * torch.where(indices == e) per expert, then the expert MLP on the gathered rows). lga_moe_group sorts the T * k
 * (token, slot) pairs by expert on the device (stable: (token, slot) order inside an expert) into a table of
 * m-tiles of bm rows (bm 64 or 256): tiles = {n_tiles, (expert, first row, rows) x n_tiles}, capacity
 * 1 + 3 * lga_moe_group_tiles(T * k, n_expert, bm) ints; x_rows[r] = token of permuted row r, y_rows[r] =
 * token * k + slot. lga_q4_gemm_swiglu_grouped computes g[r] = bf16(silu(bf16(x[x_rows[r]] W1_e^T))) *
 * bf16(x[x_rows[r]] W2_e^T) for every permuted row r in ONE launch (the experts' weights stacked with strides
 * w_stride / s_stride bytes, as lga_q4_gemv_experts); lga_q4_gemm_grouped computes y[y_rows[r]] =
 * x[x_rows ? x_rows[r] : r] W_e^T (y_rows NULL: row r). No host synchronisation: the launches are sized by the
 * table's capacity and surplus tiles exit. */
int lga_moe_group_tiles(int rows, int n_expert, int bm);
int lga_moe_group(const int32_t* expert_ids, int T, int k, int n_expert, int bm, int32_t* tiles, int32_t* x_rows,
                  int32_t* y_rows, lga_stream_t stream);
int lga_q4_gemm_swiglu_grouped(const void* x, const void* qweight1, const void* scales1, const void* qweight2,
                               const void* scales2, long long w_stride, long long s_stride, const int32_t* tiles,
                               const int32_t* x_rows, void* y, int rows, int N, int K, int group, int fmt, int bm,
                               int n_expert, lga_stream_t stream);
int lga_q4_gemm_grouped(const void* x, const void* qweight, const void* scales, long long w_stride,
                        long long s_stride, const int32_t* tiles, const int32_t* x_rows, const int32_t* y_rows,
                        void* y, int rows, int N, int K, int group, int fmt, int bm, int n_expert,
                        lga_stream_t stream);

/* -- tensor-parallel all-reduce of decode activations (generate/tp.py:73-74 `all_reduce(outs, "sum", ranks)`,
 *    the forward hook after every attention / MLP, :53,57,70) over xGMI peer memory -----------------------------
 * Each rank owns one mailbox of lga_comm_mailbox_bytes(cap) bytes from lga_comm_alloc (uncached device memory,
 * zeroed; its 64-byte IPC handle goes to the peers, which map it with lga_comm_open). lga_allreduce_bf16:
 * y[n] = bf16(sum over ranks 0..world-1, in that order, of x_r) (+ residual[n]: y = bf16(bf16(sum) + residual),
 * the Block residual add, lit_gpt/model.py:591-592), identical bits on every rank. mailboxes: host array of world
 * device pointers (index rank = this rank's own mailbox); seq_counter: 1 uint32 zeroed once, advanced by every
 * call (the same call sequence on every rank); err: bit 0 set when a peer's flag did not arrive within 5 s
 * (results invalid). n % 8 == 0, n <= cap, world <= 8. One workgroup; graph-capturable. */
size_t lga_comm_mailbox_bytes(int cap);
int lga_comm_alloc(size_t bytes, void** ptr, void* ipc_handle);
int lga_comm_open(const void* ipc_handle, void** ptr);
int lga_comm_close(void* ptr);
int lga_comm_free(void* ptr);
int lga_allreduce_bf16(const void* x, const void* residual, void* y, int n, void* const* mailboxes, int rank,
                       int world, int cap, unsigned* seq_counter, unsigned* err, lga_stream_t stream);
/* lga_comm_trace: diagnostics of the all-reduce protocol. Every later lga_allreduce_bf16 / lga_q4_gemv_allreduce
 * launch of this process records its call into buf (n_records x 16 uint64 on the device, indexed by the call's
 * sequence number): sequence, rank, entry / flags-raised / wait-done times (s_memrealtime, 100 MHz), timeout, and
 * the peers' flag words seen when the wait ended. buf = NULL switches it off. Not part of the reference interface. */
int lga_comm_trace(void* buf, int n_records);
/* The row-parallel decode Linear and its all-reduce in ONE launch (generate/tp.py:53,57,70 hook the reduction on
 * attn.proj / mlp.proj; lit_gpt/model.py:591-592 adds the residual): y (N) = lga_allreduce_bf16 of
 * lga_q4_gemv(x, W, bias) over the ranks (+ residual), bit for bit — each workgroup pushes its partial rows into
 * every rank's mailbox, the last-arriving workgroup of the rank raises the flags, waits for the peers and sums in
 * rank order. Same mailboxes / sequence counter / error word as lga_allreduce_bf16 (calls of the two may be mixed);
 * arrive_counter: 576 uint32 (9 counters at a 256-B stride; 640 with the tagged form's) zeroed once (re-armed by the kernel). N % 8 == 0, N <= cap. Graph-capturable. */
int lga_q4_gemv_allreduce(const void* x, const uint8_t* qweight, const void* scales, const void* bias,
                          const void* residual, void* y, int N, int K, int group, int fmt, void* const* mailboxes,
                          int rank, int world, int cap, unsigned* seq_counter, unsigned* arrive_counter,
                          unsigned* err, lga_stream_t stream);
/* The same call in the tagged protocol (generate/tp.py:73-74 on multi-GPU ranks): every workgroup pushes its rows as
 * 8-byte {bf16 pair, call sequence} granules into every rank's mailbox and polls its own rows from every rank — no
 * arrival counters, flags or last-arriver sum; identical result bits. arrive_counter: 640 uint32 (words 576 / 608:
 * the launch's arrivals and the rank's call count the sequence derives from, zeroed once); seq_counter unused. The grid need not be
 * co-resident (a workgroup waits only for other ranks). Same mailboxes: lga_comm_mailbox_bytes covers both regions. */
int lga_q4_gemv_allreduce_tagged(const void* x, const uint8_t* qweight, const void* scales, const void* bias,
                                 const void* residual, void* y, int N, int K, int group, int fmt,
                                 void* const* mailboxes, int rank, int world, int cap, unsigned* seq_counter,
                                 unsigned* arrive_counter, unsigned* err, lga_stream_t stream);

/* -- greedy sampling (generate/base.py:30-47 at temperature 0): lowest index among the maxima; optionally
 *    writes the token (int32) and advances *pos_inout by one (generate/base.py:92) -------------------------- */
int lga_argmax(const void* logits, int n, int64_t* out_idx, int32_t* token_out, int64_t* pos_inout,
               lga_stream_t stream);
/* lga_argmax, then the same launch gathers row `token` of the embedding table (vocab x n_embd bf16) into emb_out
 * (n_embd bf16): the next decode step's transformer.wte(idx) (lit_gpt/model.py:515, an nn.Embedding gather),
 * bit-identical to lga_embedding of the token — one launch per step fewer. */
int lga_argmax_embed(const void* logits, int n, int64_t* out_idx, int32_t* token_out, int64_t* pos_inout,
                     const void* table, int n_embd, int vocab, void* emb_out, lga_stream_t stream);
/* lga_q4_gemv_argmax_embed: the greedy decode step's head in ONE launch — optional fused RMSNorm (ln_f), the 4-bit
 * lm_head GEMV (model.py:519; logits (N) bf16 still written), argmax (generate/base.py:30-41 at temperature 0,
 * torch.argmax order: NaN first, ties to the lowest index) and lga_argmax_embed's bookkeeping (token_out, out_idx,
 * *pos_inout += 1, the token's row of table into emb_out). Bit-identical to lga_q4_gemv + lga_argmax_embed.
 * work: lga_q4_gemv_argmax_work_bytes(N, K) bytes, zeroed once (its counters re-arm). K <= 4096. */
size_t lga_q4_gemv_argmax_work_bytes(int N, int K);
int lga_q4_gemv_argmax_embed(const void* x, const uint8_t* qweight, const void* scales, const void* norm_weight,
                             float norm_eps, void* logits, int N, int K, int group, int fmt, void* work,
                             int64_t* out_idx, int32_t* token_out, int64_t* pos_inout, const void* table, int C, int V,
                             void* emb_out, lga_stream_t stream);

/* -- temperature sampling (generate/base.py:30-41 with top_k and temperature > 0: torch.topk, scatter into -inf,
 *    softmax(logits / temperature) in the logits' dtype, torch.multinomial(probs, 1)) in ONE launch --------------
 * logits: n (<= 65536) bf16. Keeps the top_k (1..1024) largest (NaN largest, ties lowest index first),
 * x = bf16(v / temperature), p = bf16(exp(x - max) / sum); the token is the first kept index (in index order) whose
 * running fp32 sum of p divided by the total reaches u (torch's CPU inverse CDF). u = *uniform when uniform is
 * given, else a counter-based hash of (seed, *counter) in (0, 1), and *counter advances by one (device state: the
 * launch replays in a graph). Then lga_argmax's bookkeeping (out_idx, token_out, *pos_inout += 1) and, with emb_out,
 * lga_argmax_embed's row gather. kept_out (top_k int32) / probs_out (top_k bf16), optional: the kept indices in
 * index order and their probabilities. */
int lga_sample_topk(const void* logits, int n, int top_k, float temperature, const float* uniform,
                    unsigned long long seed, unsigned long long* counter, int64_t* out_idx, int32_t* token_out,
                    int64_t* pos_inout, const void* table, int n_embd, int vocab, void* emb_out, int32_t* kept_out,
                    void* probs_out, lga_stream_t stream);

/* -- fp32 forward (the reference's --precision 32-true, generate/base.py:132; BASELINE config 1 pythia-160m fp32):
 *    float32 weights and activations, no bf16 rounding; plumbing-sized kernels (csrc/fp32.hip) -------------- */
/* y (M, N) = x (M, K) . w (N, K)^T (+ bias[N]) (+ residual (M, N)) — F.linear (lit_gpt/model.py:519,619,656,699-702) */
int lga_f32_linear(const float* x, const float* w, const float* bias, const float* residual, float* y, int M, int N,
                   int K, lga_stream_t stream);
/* torch.nn.LayerNorm over rows of n (config.py:137-144): two-pass mean / biased variance, (x - mean) * rstd * w + b */
int lga_f32_layernorm(const float* x, const float* w, const float* b, float* y, int rows, int n, float eps,
                      lga_stream_t stream);
/* F.gelu (exact erf, or tanh when approximate_tanh) — GptNeoxMLP (model.py:699-702) */
int lga_f32_gelu(const float* a, float* y, long n, int approximate_tanh, lga_stream_t stream);
/* y = a + b (the Block residual adds, model.py:584-593) */
int lga_f32_add(const float* a, const float* b, float* y, long n, lga_stream_t stream);
/* lga_rope_kv_append in fp32: apply_rope on the first rope_n_elem dims (model.py:641-644, 767-773) + KVCache.forward
 * (:788-795); caches (G, max_seq, hs) fp32 */
int lga_f32_rope_kv_append(const float* qkv, float* q_out, float* k_cache, float* v_cache, const int64_t* cache_pos,
                           const int64_t* rope_pos, const float* cos, const float* sin, int rope_rows, int T,
                           int n_head, int n_query_groups, int head_size, int rope_n_elem, int max_seq,
                           lga_stream_t stream);
/* SDPA (model.py:651, 658-665) in fp32: q (T, H, hs), caches (G, max_seq, hs), query t attends keys 0..input_pos[t];
 * y (T, H*hs). head_size <= 256, max_seq <= 32768. */
int lga_f32_attention(const float* q, const float* k_cache, const float* v_cache, const int64_t* input_pos, float* y,
                      int T, int n_head, int n_query_groups, int head_size, int max_seq, float scale,
                      lga_stream_t stream);
/* lga_argmax over fp32 logits (generate/base.py:30-47 at temperature 0) */
int lga_argmax_f32(const float* logits, int n, int64_t* out_idx, int32_t* token_out, int64_t* pos_inout,
                   lga_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* LITGPT_AMD_H */
