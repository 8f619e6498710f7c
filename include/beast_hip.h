/*
 * beast_hip.h -- C-ABI of libbeast_hip.so, the MI355X (gfx950) hot path of BEAST.
 *
 * The reference (Dont4rootMe/beast_tokenizer) has no native boundary: its
 * "plugin point" is the mp_pytorch UniformBSpline object, beast/utils.py and the
 * HF `tokenizers` BpeTrainer.  Each entry point below replaces one of those call
 * sites (cited per function) and is what a ctypes / cffi binding of the
 * reference would bind.
 *
 * Conventions
 *   - Plain C types only.  All pointers are DEVICE pointers unless named host_*.
 *   - The caller allocates every input, output and workspace buffer.
 *   - Every call is stream-ordered on `stream` (a hipStream_t passed as void*);
 *     nothing synchronises the device except where a function says so.
 *   - Return 0 on success or a negative BEAST_E_* code; beast_last_error()
 *     returns a thread-local message for the last failure.  No C++ exception
 *     crosses this boundary.
 *   - Layouts: params are [B][D*N] "(d n)" order, tokens are [B][N*D] "(n d)"
 *     order, exactly as beast/beast_bspline_tokenizer.py:418-422 produces them.
 *     The DoF order d is joint_indices ++ gripper_indices (:70, :414); the
 *     first n_joint DoFs use basis kind 0 (degree p), the rest kind 1
 *     (degree 0 gripper basis, :88-96).
 */
#ifndef BEAST_HIP_H
#define BEAST_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BEAST_OK 0
#define BEAST_E_INVALID (-1)     /* bad argument (maps to ValueError)          */
#define BEAST_E_HIP (-2)         /* HIP runtime / launch failure (RuntimeError) */
#define BEAST_E_UNSUPPORTED (-3) /* shape outside the kernels' envelope       */
#define BEAST_E_WORKSPACE (-4)   /* workspace too small                       */

#define BEAST_ABI_VERSION 1

int beast_abi_version(void);
const char* beast_last_error(void);

/* Process-wide tuning / test options.  BEAST_OPT_GENERIC_KERNELS = 1 makes encode and
 * reconstruct use their runtime-shape kernels even where a shape-specialised kernel
 * exists (the BEAST defaults T = 50, N = 10, D = 7 / 14); results are identical.
 * BEAST_OPT_BLOCK_WAVES = 4 or 7 forces the workgroup width of the specialised 14-DoF
 * kernels, 8 forces the per-trajectory kernels (16 waves since round 6; 0 = chosen by batch size); results are
 * identical.
 * BEAST_OPT_MERGE_LDS_MIN = n: BPE merges of pairs counted >= n privatise their pair-count deltas
 * in LDS (default 4096; below, global atomics); results are identical.
 * BEAST_OPT_BPE_ENCODE_MODE = m (tests, measurements): beast_bpe_encode_rows' per-word merge by
 * rounds (0, the default) or by HF's min-heap (1); m + 2 also launches one workgroup per 4 rows
 * instead of only the resident ones.  Results are identical.
 * BEAST_OPT_BPE_DEDUP_KEY_BITS = k (tests): beast_bpe_encode_rows_words keeps only k bits of its
 * 32-bit word hashes, so different words share hashes; the code-point compare behind every hash
 * match keeps them apart (same ids).
 * BEAST_OPT_BPE_TRAIN_HOST_LOOP = 1 (tests): beast_bpe_train runs the host-driven loop at any Vt;
 * 2 reruns it after the batched loop as a string-hash collision would.  Results are identical.
 * Options are process-wide and not synchronised: set them before launching, not concurrently. */
#define BEAST_OPT_GENERIC_KERNELS 1
#define BEAST_OPT_BLOCK_WAVES 2
#define BEAST_OPT_MERGE_LDS_MIN 3
#define BEAST_OPT_BPE_ENCODE_MODE 5
#define BEAST_OPT_BPE_DEDUP_KEY_BITS 6
#define BEAST_OPT_BPE_TRAIN_HOST_LOOP 7
int beast_set_option(int option, int value);
/* the option's current value (BEAST_E_INVALID for an unknown option) */
int beast_get_option(int option);

/* ---------------------------------------------------------------- H1/H2 ---
 * Replaces UniBSplineBasis.basis (MP_lite_PyTorch/mp_pytorch/basis_gn/
 * uni_bspline_basis.py:59-113) with LinearPhaseGenerator.phase
 * (phase_gn/linear_phase.py:22-24): basis_out[i][n] = B_{n,degree}(clip((t_i -
 * delay)/tau, 0, 1)) by the same Cox-de Boor recursion, same fp32 op order.
 * knots: [n_knots] with n_knots == degree + 1 + num_basis.  degree <= 8. */
int beast_bspline_basis_f32(const float* times, int64_t n_times, float tau, float delay,
                            const float* knots, int n_knots, int degree, int num_basis,
                            float* basis_out, void* stream);

/* Ridge projection P = (Phi^T Phi + reg I)^-1 Phi^T in float64: the closed form
 * of UniformBSpline.learn_mp_params_from_trajs (mp/uni_bspline.py:539-586) for
 * init/end condition order 0, where the block-diagonal system of
 * basis_multi_dofs (basis_gn/uni_bspline_basis.py:349-356) decouples per DoF.
 * Written zero-padded as proj_out[16][Tp], Tp = round_up(T, 4) (the MFMA A-operand
 * layout of beast_encode_f32).  One workgroup; N <= 16. */
int beast_bspline_projection_f64(const float* basis, int T, int N, double reg, double* proj_out,
                                 void* stream);

/* ------------------------------------------------------------- H4 + H5 ---
 * Replaces BEASTBsplineTokenizer.encode (beast/beast_bspline_tokenizer.py:
 * 399-428) -> learn_mp_params_from_trajs + clamp + continuous_to_discrete
 * (beast/utils.py:4-17) + rearrange + LLM offset, as ONE fused kernel.
 *   traj[b*sb + t*st + dof_src[d]*sd]  fp32 input, element strides
 *   row_elems   size of the input's last dim (for the contiguous fast path)
 *   proj        [2][16][Tp] fp32 zero-padded projections (kind 0 joint, kind 1
 *               gripper): the round-to-nearest fp32 image of the float64 output of
 *               beast_bspline_projection_f64, converted once per time grid
 *   params_out  [B][D*N] fp32 unclamped fit (params_dict['params']); nullable
 *   tokens_out  [B][N*D] int64 = round_half_even(clamp01((clamp(p)-wmin)/max(wmax-wmin,1e-8))*(vocab-1))
 *               + tok_offset; nullable.  vocab <= 0 disables quantisation.
 * Constraints: N <= 16, T <= 256, D <= 64. */
int beast_encode_f32(const float* traj, int64_t B, int T, int64_t sb, int64_t st, int64_t sd, int row_elems,
                     int D, int n_joint, const int32_t* dof_src, const float* proj, int N,
                     const float* w_min, const float* w_max, int vocab, int64_t tok_offset,
                     float* params_out, int64_t* tokens_out, void* stream);

/* Params-only fit of a LIST of batches in one launch (fit_parameters, reference :181-220,
 * which fits every dataloader batch then takes quantiles): batch i's rows start at the
 * device pointer traj_list[i] (traj_list itself is a device array of nbatch pointers, each
 * 16-byte aligned), every batch has rows_per_batch (a multiple of 8) contiguous rows of
 * [T][row_elems] fp32; params_out [nbatch * rows_per_batch][D*N] (d n).  Same kernel and
 * arithmetic as beast_encode_f32, so params are bitwise those of per-batch calls. */
int beast_encode_list_f32(const float* const* traj_list, int nbatch, int64_t rows_per_batch, int T, int row_elems,
                          int D, int n_joint, const int32_t* dof_src, const float* proj, int N, float* params_out,
                          void* stream);

/* Quantise-only epilogue of the above for already-fitted params [B][D*N] (d n):
 * used by encode(update_bounds=True) after the bounds move (:415-420).
 * mode 0: tokens_out int64 [B][N*D] (continuous_to_discrete + offset);
 * mode 1: ntok_out fp32 [B][N*D] = normalize_tensor (beast/utils.py:29-35),
 *         the encode_continuous path (:430-450). */
int beast_quantize_f32(const float* params, int64_t B, int D, int N, const float* w_min, const float* w_max,
                       int vocab, int64_t tok_offset, int mode, int64_t* tokens_out, float* ntok_out, void* stream);

/* ------------------------------------------------------------- H6 - H8 ---
 * Replaces BEASTBsplineTokenizer.decode + reconstruct_traj (beast/
 * beast_bspline_tokenizer.py:483-536) -> discrete_to_continuous (beast/
 * utils.py:20-26), optional init_p overwrite of coefficient 0 of the joint
 * DoFs (:505-510), UniformBSpline.get_traj_pos (mp/uni_bspline.py:114-177)
 * and the scatter to joint/gripper columns (:520-534).
 *   tokens      [B][N*D] int64 (tok_offset is SUBTRACTED first)
 *   basis       [2][T_out][N] fp32 per kind; batch stride basis_sb (0 = shared)
 *   dof_dst     [D] output column of each DoF; pos_out [B][T_out][num_dof_out]
 *   init_p      nullable [B] rows of stride init_p_sb; init_p_src[d] column for
 *               joint DoF d (< n_joint)
 *   params_out  nullable [B][D*N] decoded params (= decode()); pos_out nullable.
 *   ntokens     nullable: when set, fp32 normalised tokens [B][N*D] in [-1, 1] are
 *               read instead of `tokens` and mapped back by denormalize_tensor
 *               (beast/utils.py:38-44): the reconstruct_traj_continuous path (:538-582). */
int beast_reconstruct_f32(const int64_t* tokens, int64_t B, int D, int n_joint, int N, int vocab,
                          int64_t tok_offset, const float* w_min, const float* w_max,
                          const float* basis, int64_t basis_sb, int T_out,
                          const int32_t* dof_dst, int num_dof_out,
                          const float* init_p, int64_t init_p_sb, const int32_t* init_p_src,
                          float* params_out, float* pos_out, const float* ntokens, void* stream);

/* ---------------------------------------------------- §8f rank 4: conditions ---
 * init_cond_order / end_cond_order != 0 (init_order in 0..2, end_order in -1..2, not both 0).
 * beast_cond_fixed_f32 replaces the per-fit condition step of UniBSpline.learn
 * (MP_lite_PyTorch/mp_pytorch/mp/uni_bspline.py:499-550 calling compute_init_params /
 * compute_end_params, basis_gn/uni_bspline_basis.py:192-301): for trajectories traj
 * [B][T][*] (element strides sb, st, sd) and the joint DoFs joint_idx[dj], with
 * dt = times[1] - times[0] and the knot steps knots[1+degree] - knots[1] /
 * knots[n_ctrl-1+degree] - knots[n_ctrl-1] of the joint spline (n_ctrl control points):
 *   init_pos, init_vel [B][dj], params_init [B][dj][init_order]   (init_order > 0)
 *   end_pos, end_vel [B][dj], params_end [B][dj][|end_order|]     (end_order != 0)
 * in the reference's fp32 op order.  T >= 2.
 * beast_cond_add_f32 replaces the fixed control points' part of UniBSpline.get_traj_pos
 * (uni_bspline.py:126-166): pos [B][T][D] (contiguous, the fitted columns' positions from
 * beast_reconstruct_f32) gains, at the joint DoFs, sum_k full_basis[t][k] * fixed[k] (+ init_pos
 * when init_order > 0) over the fixed columns k (the first init_order, the last |end_order|;
 * end order -1 subtracts params_end from column n_ctrl-2).  full_basis [T][n_ctrl] with
 * full_sb = 0, or per trajectory [B][T][n_ctrl] with full_sb = T * n_ctrl. */
int beast_cond_fixed_f32(const float* traj, int64_t B, int T, int64_t sb, int64_t st, int64_t sd,
                         const int32_t* joint_idx, int dj, const float* times, const float* knots, int degree,
                         int n_ctrl, float tau, int init_order, int end_order, float* init_pos, float* init_vel,
                         float* end_pos, float* end_vel, float* params_init, float* params_end, void* stream);
int beast_cond_add_f32(float* pos, int64_t B, int T, int D, const int32_t* joint_idx, int dj,
                       const float* full_basis, int64_t full_sb, int n_ctrl, int init_order, int end_order,
                       const float* params_init, const float* params_end, const float* init_pos, void* stream);

/* ------------------------------------------------------------------ H13 ---
 * Column min / max with NaN propagation (torch.min/max(dim=0)), used by
 * update_weights_bounds / update_weights_bounds_per_batch (:362-389).
 * workspace >= beast_colminmax_workspace_bytes(rows, cols). */
size_t beast_colminmax_workspace_bytes(int64_t rows, int cols);
int beast_colminmax_f32(const float* x, int64_t rows, int cols, int64_t row_stride, float* out_min,
                        float* out_max, void* workspace, size_t ws_bytes, void* stream);

/* Exact per-column quantiles with numpy 'linear' semantics in float32
 * (np.quantile(params, q, axis=0), :213-214) by radix select on order-preserving keys:
 * radix_bits 11 (three passes: 11/11/10 bits) or 7 (four passes: 11/7/7/7 bits; smaller histograms
 * to all-reduce for one more pass over the keys).  Multi-GPU: call
 * prepare, then for pass in 0 .. beast_quantile_passes(radix_bits) - 1 { hist; all-reduce(SUM,
 * uint32) of the first beast_quantile_hist_count(pass, ...) elements at beast_quantile_hist_ptr;
 * select }, then finalize (every rank selects the same order statistics).  n_total = rows summed
 * over all ranks (< 2^32).  n_q <= 4 (host_q). */
size_t beast_quantile_workspace_bytes(int64_t rows, int cols, int n_q);
int beast_quantile_prepare(const float* x, int64_t rows, int cols, int64_t row_stride, int64_t n_total,
                           int n_q, const float* host_q, void* workspace, size_t ws_bytes, void* stream);
uint32_t* beast_quantile_hist_ptr(void* workspace, int cols, int n_q);
int beast_quantile_passes(int radix_bits);
int64_t beast_quantile_hist_count(int pass, int cols, int n_q, int radix_bits);
/* prepare over a list of row-major segments instead of one matrix (fit_parameters' per-batch
 * params without a concatenation): seg_table = device array of nseg {const float* ptr;
 * int64_t first_row; int64_t row_stride} (24 B each, first_row ascending from 0), rows = the
 * total, max_seg_rows = the largest segment. */
int beast_quantile_prepare_segments(const void* seg_table, int nseg, int64_t max_seg_rows, int64_t rows, int cols,
                                    int64_t n_total, int n_q, const float* host_q, void* workspace, size_t ws_bytes, void* stream);
int beast_quantile_hist(int pass, int64_t rows, int cols, int n_q, int radix_bits, void* workspace, void* stream);
int beast_quantile_select(int pass, int cols, int n_q, int radix_bits, void* workspace, void* stream);
int beast_quantile_finalize(int cols, int n_q, void* workspace, float* out, void* stream);
/* single-GPU convenience: all of the above. out [n_q][cols]. */
int beast_quantile_f32(const float* x, int64_t rows, int cols, int64_t row_stride, int n_q, const float* host_q,
                       float* out, void* workspace, size_t ws_bytes, void* stream);

/* ------------------------------------------------------------ H9 - H12 ---
 * Byte-level BPE training, replacing HF tokenizers' BpeTrainer::do_train as
 * driven by FIGBPE (beast/beast_bpe_trainer.py:61-98).  Tokens are int64 code
 * points (bins); a sequence is tokens[seq_off[s] .. seq_off[s+1]). */
int beast_i64_minmax(const int64_t* x, int64_t n, int64_t* out2, void* stream);
/* present[x - min_tok] = 1 for every token (n_cp = max-min+1); multi-GPU: all-reduce MAX */
int beast_bpe_cp_presence(const int64_t* tok, int64_t n, int64_t min_tok, uint8_t* present, int64_t n_cp,
                          void* stream);
/* GPT-2 ByteLevel pre-tokenisation, pass 1: words and byte-symbols per sequence.
 * cls_lut[cp] in {0 other, 1 letter, 2 number, 3 whitespace}, cp < lut_n. */
int beast_bpe_pretok_count(const int64_t* tok, const int64_t* seq_off, int64_t n_seq, int64_t min_tok,
                           const uint8_t* cls_lut, int64_t lut_n, int64_t* words_per_seq,
                           int64_t* syms_per_seq, void* stream);
/* exclusive scan: out[0..n] (out[n] = total). workspace >= beast_scan_workspace_bytes(n) */
size_t beast_scan_workspace_bytes(int64_t n);
int beast_exclusive_scan_i64(const int64_t* in, int64_t* out, int64_t n, void* workspace, void* stream);
/* pass 2: emit byte symbols as vocab ids (byte2id[256]) and word extents. */
int beast_bpe_pretok_emit(const int64_t* tok, const int64_t* seq_off, int64_t n_seq, int64_t min_tok,
                          const uint8_t* cls_lut, int64_t lut_n, const int64_t* word_off,
                          const int64_t* sym_off, const uint16_t* byte2id, uint16_t* sym,
                          uint32_t* wstart, uint32_t* wlen, void* stream);
/* pair table [Vt][Vt] uint32 += word count for each adjacent pair (BpeTrainer::count_pairs).
 * n_sym: every symbol id is < n_sym (the setup vocabulary); small n_sym count in LDS. */
int beast_bpe_count_pairs(const uint16_t* sym, const uint32_t* wstart, const uint32_t* wlen,
                          const uint32_t* wcount, int64_t n_words, uint32_t* table, int Vt, int n_sym,
                          void* stream);
/* sig[w] = OR over word w's symbols x of two bits of x (a 64-bit Bloom mask, csrc/bpe_common.h
 * sig_bit).  The merges use it to skip words that cannot contain a pair without reading their
 * symbols, and keep it current for the words they rewrite. */
int beast_bpe_word_signatures(const uint16_t* sym, const uint32_t* wstart, const uint32_t* wlen, int64_t n_words,
                              uint64_t* sig, void* stream);

/* -- the merge loop (csrc/bpe_loop.hip), replacing the loop of HF BpeTrainer::do_train as called
 * from beast/beast_bpe_trainer.py:61-74.  Two forms over the same words:
 *
 * Host-driven, one merge per call (vocabularies above 4096, the host fallback on a string-hash
 * collision, the per-merge all-reduce form):
 * max over table[x][y], x,y < vcur, of (count << 32 | ~(x*Vt+y)) (0 if the table is empty)
 * into ws[2 + (call & 1)], where call = 0, 1, 2, ... numbers the calls on this workspace
 * (each call zeroes the other slot for the next one: no memset per call).  Incremental:
 * ws caches each row's best; a row is rescanned only when beast_bpe_apply_argmax changed it
 * -- any other table write needs a fresh zero-filled ws.
 * ws: beast_bpe_argmax_workspace_bytes(Vt), zero-filled once before call 0. */
size_t beast_bpe_argmax_workspace_bytes(int Vt);
int beast_bpe_argmax(const uint32_t* table, int Vt, int vcur, uint64_t* ws, int call, void* stream);
/* Merge (a,b)->new_id in every word, left to right, non-overlapping (HF Word::merge);
 * HF's pair-count changes, per word times wcount (NULL = 1):
 * [0]: (x,a)  [1]: (x,new)  [2]: (b,y)  [3]: (new,y).
 * are accumulated into deltas[4][Vt] int32 (multi-GPU: all-reduce them, then
 * beast_bpe_apply_argmax).  sig: beast_bpe_word_signatures.  pair_count: the pair's count from
 * beast_bpe_argmax (a hint choosing LDS-privatised or direct delta atomics). */
int beast_bpe_merge(uint16_t* sym, const uint32_t* wstart, uint32_t* wlen, const uint32_t* wcount,
                    int64_t n_words, int a, int b, int new_id, const uint32_t* tlen, int max_token_length,
                    int32_t* deltas, int Vt, uint64_t* sig, int64_t pair_count, void* stream);
/* The step after a merge, fused with the next argmax: table += deltas (deltas consumed are
 * zeroed), table[a][b] = 0 (merged pair retired), tlen[new_id] = tlen[a] + tlen[b]; then the
 * argmax of beast_bpe_argmax (same ws, next call index) over x, y < vcur (vcur counting new_id). */
int beast_bpe_apply_argmax(uint32_t* table, int32_t* deltas, int Vt, int vcur, int a, int b, int new_id,
                           uint32_t* tlen, uint64_t* ws, int call, void* stream);

/* Device-driven, batched (the default): merges are decided on the GPU, several per pass and
 * exactly HF's sequence -- each pass takes the table's top pairs in HF order while none chains
 * onto a taken one (its right symbol a taken left symbol, or its left a taken right), no taken
 * pair was a self-pair or re-used an id, and no taken row's next key ranks above it
 * (csrc/bpe_loop.hip, "batched merges", has the proof); stop rules: vocab_size reached, count below min_frequency, log full.
 * Ids of new strings come from a (64-bit string hash, byte length) table of the vocabulary
 * (HF's id reuse); the host replays the log against the real strings.
 * tok_hash / tok_pow: per initial token, h = sum bytes[i] * P^(n-1-i) and P^n (mod 2^64) of its
 * UTF-8 string; tlen its length in HF units (characters of the byte-level string), max_tlen
 * the largest.  beast_bpe_loop_state returns device pointers to the state {int32 active, vcur,
 * n_merges, ...} and the log [max_merges][4] int32 {a, b, nid, reused} for the host to read. */
size_t beast_bpe_loop_workspace_bytes(int Vt, int max_merges);
int beast_bpe_loop_init(void* ws, size_t ws_bytes, int Vt, int max_merges, int n_tokens, int vocab_size,
                        int min_frequency, const uint64_t* tok_hash, const uint64_t* tok_pow, const uint32_t* tlen,
                        int max_tlen, void* stream);
int beast_bpe_loop_state(const void* ws, int Vt, int max_merges, const void** state, const void** log);
/* n_steps passes of (merge the decided batch over every word, apply + rank + decide the next),
 * two launches each; passes after the loop stopped are no-ops.  max_batch (2, 4 or 8) caps a
 * pass.  argws: beast_bpe_argmax_workspace_bytes(Vt), zero-filled; batch_ws:
 * beast_bpe_batch_workspace_bytes(Vt).  flags: BEAST_BPE_BATCH_INIT ranks every row and decides
 * the first batch before the passes (first call after beast_bpe_loop_init); _NO_MERGE / _NO_APPLY
 * leave out one launch of each pass -- the sharded form: each rank holds a shard of the words,
 * its merge launch writes the pair-count changes into deltas [beast_bpe_batch_delta_count(Vt)]
 * int32 (zero-filled once) instead of the table, the caller all-reduces (SUM) them, and the apply
 * launch adds them to every rank's identical table (deltas NULL: one GPU, the changes go straight
 * into the table).  apps (nullable, accounting): apps[m] += the pair occurrences merge m
 * rewrote in the distinct words.  Vt <= 4096. */
#define BEAST_BPE_BATCH_INIT 1
#define BEAST_BPE_BATCH_NO_MERGE 2
#define BEAST_BPE_BATCH_NO_APPLY 4
size_t beast_bpe_batch_workspace_bytes(int Vt);
size_t beast_bpe_batch_delta_count(int Vt);
int beast_bpe_loop_batch(void* ws, int Vt, int max_merges, int n_steps, int max_batch, int flags, uint16_t* sym,
                         const uint32_t* wstart, uint32_t* wlen, const uint32_t* wcount, int64_t n_words,
                         uint32_t* tlen, int max_token_length, uint64_t* sig, uint32_t* table, uint64_t* argws,
                         void* batch_ws, size_t batch_ws_bytes, int vocab_size, int32_t* deltas, uint32_t* apps,
                         void* stream);
/* One-call training (round 4; SURVEY.md §8b's beast_bpe_train): FIGBPE.fit_from_sequences
 * (beast/beast_bpe_trainer.py:76-98 -> :61-74, HF BpeTrainer(vocab_size, min_frequency,
 * special_tokens, initial_alphabet = chr(0 .. max - min), max_token_length).train_from_iterator
 * over the strings "".join(map(chr, seq - min))) on one GPU, the steps above in order: min /
 * max, presence, alphabet (special tokens, then byte-level chars and the initial alphabet by
 * code point), pretok count / scan / emit, dedup, repack, signatures, pair table, the batched
 * loop, the host replay of its log.  tokens / seq_off [n_seq + 1] / cls_lut [lut_n >= max - min
 * + 1] (beast_tokenizer_amd/pretok.py class_lut) are DEVICE pointers; special_tokens n_special
 * NUL-terminated UTF-8 strings (host).  Outputs (HOST): the token range, the vocabulary as UTF-8
 * strings in id order (out_vocab_bytes[out_vocab_off[i] .. out_vocab_off[i+1])), the merges as
 * id pairs out_merges[2m], [2m+1] (merge m's token is their concatenation, the next new id
 * unless the string already had one).  Capacities: max_vocab >= max(vocab_size, alphabet),
 * max_merges_out >= vocab_size - alphabet (checked up front), vocab_bytes_cap >= the strings'
 * bytes (known only after training).  When an output is too small the call returns
 * BEAST_E_WORKSPACE with the required sizes in *out_n_vocab, *out_n_merges and out_vocab_off[0]
 * (vocabulary bytes); retry with those.  Synchronises the stream.  Vt <= 4096 runs the batched
 * device loop; 4096 < Vt <= 32768 the host-driven one (beast_bpe_argmax / _merge / _apply_argmax,
 * one host read per merge), as does a rerun after a full merge log or a 64-bit string-hash
 * collision of the batched loop; BEAST_E_UNSUPPORTED above 32768 (the dense pair table).  One
 * GPU; beast_bpe_train_comm below is the multi-rank form. */
int beast_bpe_train(const int64_t* tokens, const int64_t* seq_off, int64_t n_seq, const uint8_t* cls_lut,
                    int64_t lut_n, int vocab_size, int min_frequency, int max_token_length,
                    const char* const* special_tokens, int n_special, int64_t* out_min_token,
                    int64_t* out_max_token, char* out_vocab_bytes, size_t vocab_bytes_cap, int64_t* out_vocab_off,
                    int max_vocab, int* out_n_vocab, int32_t* out_merges, int max_merges_out, int* out_n_merges,
                    void* stream);

/* ---- The library's own RCCL communicator (round 5; SURVEY.md §8b's beast_comm_init / destroy
 * and the comm argument of the training call), for a multi-GPU caller without torch.distributed.
 * RCCL is bound at run time (librccl.so.1; inside a torch process the copy torch mapped), so the
 * library loads without it; every entry point returns BEAST_E_UNSUPPORTED when it is absent.
 * One process per GPU: rank 0 makes an id (beast_comm_unique_id, beast_comm_id_bytes() bytes),
 * the caller hands it to every rank, each calls beast_comm_init_rank with its own device.
 * beast_comm_init is the single-process form (one handle per listed device, out[ndev]). */
typedef struct beast_comm beast_comm;
#define BEAST_DT_U8 0
#define BEAST_DT_I32 1
#define BEAST_DT_U32 2
#define BEAST_DT_I64 3
#define BEAST_DT_U64 4
#define BEAST_DT_F32 5
#define BEAST_DT_F64 6
#define BEAST_OP_SUM 0
#define BEAST_OP_MIN 1
#define BEAST_OP_MAX 2
size_t beast_comm_id_bytes(void);
int beast_comm_unique_id(void* id_out);
int beast_comm_init_rank(int world, int rank, const void* id, int device, beast_comm** out);
/* The single-process form's collectives (beast_comm_init with ndev > 1, one host thread driving
 * every handle) must be issued between beast_comm_group_start() and beast_comm_group_end(), as
 * ncclGroupStart / ncclGroupEnd require; otherwise drive each handle from its own host thread.
 * beast_bpe_train_comm issues collectives of its own: call it from one host thread per handle. */
int beast_comm_init(int ndev, const int* devs, beast_comm** out);
int beast_comm_group_start(void);
int beast_comm_group_end(void);
/* n virtual ranks on one device (SURVEY.md §4.3's "N virtual ranks on one device"; tests and
 * rehearsal on a one-GPU box): out[n] handles of a world of n, each driven by its own host thread.
 * Every collective synchronises the caller's stream and meets the other ranks in host memory
 * (rank-ordered reductions), so the library's multi-rank code paths run where RCCL cannot form a
 * world > 1.  A rank that does not arrive within 120 s fails the collective on every rank. */
int beast_comm_init_virtual(int n, int device, beast_comm** out);
int beast_comm_destroy(beast_comm* comm);
int beast_comm_info(const beast_comm* comm, int* world, int* rank, int* device);
/* §8e's reductions on device buffers (in place when send == recv), stream-ordered: the running
 * bounds (MIN / MAX over [D*N] f32, beast/beast_bspline_tokenizer.py:362-389), the quantile
 * histograms and BPE pair tables (SUM). */
int beast_comm_allreduce(beast_comm* comm, const void* send, void* recv, int64_t count, int dtype, int op,
                         void* stream);
int beast_comm_allgather(beast_comm* comm, const void* send, void* recv, int64_t count, int dtype, void* stream);
/* rank r's counts[r] elements at recv + displs[r] on every rank; counts / displs HOST [world],
 * equal on every rank */
int beast_comm_allgatherv(beast_comm* comm, const void* send, void* recv, const int64_t* counts,
                          const int64_t* displs, int dtype, void* stream);
/* beast_bpe_train over every rank's shard of the sequences (SURVEY.md §8b's comm argument;
 * FIGBPE.fit_from_sequences with process_group, beast/beast_bpe_trainer.py:61-98): the token
 * range is all-reduced (MIN / MAX), the code-point presence (MAX), each rank pre-tokenises and
 * deduplicates its shard, the distinct words x counts are all-gathered once (rank order) and
 * every rank runs the batched loop on the union -- bpe_train.py's replicated form, no per-pass
 * collective (replicate != 0).  replicate == 0 is the sharded form: every rank keeps its own
 * words, the pair table is SUM-reduced once and each pass's pair-count changes are SUM-reduced
 * between its merge and apply launches (the host-driven loop: each merge's), so the words of
 * no single GPU need to hold the corpus.  Every rank returns the same vocabulary and merges; a
 * shard may be empty (n_seq 0, or sequences without tokens), in either form.  All ranks must call it with the same options.  A failure
 * on one rank (an allocation, a launch, a shard over 2^32 symbols) is agreed over the communicator
 * before the next collective (the status all-reduced with MAX), so every rank returns an error
 * together: the failing rank its own, the others its code with a message naming the cause.
 * comm == NULL is beast_bpe_train. */
int beast_bpe_train_comm(const int64_t* tokens, const int64_t* seq_off, int64_t n_seq, const uint8_t* cls_lut,
                         int64_t lut_n, int vocab_size, int min_frequency, int max_token_length,
                         const char* const* special_tokens, int n_special, int64_t* out_min_token,
                         int64_t* out_max_token, char* out_vocab_bytes, size_t vocab_bytes_cap, int64_t* out_vocab_off,
                         int max_vocab, int* out_n_vocab, int32_t* out_merges, int max_merges_out, int* out_n_merges,
                         beast_comm* comm, int replicate, void* stream);
/* Distinct words (HF BpeTrainer trains on word -> count): every word of >= 2 symbols is
 * matched by content (hash tag + symbol-by-symbol compare, so collisions never merge
 * different words); out_* get one entry per distinct word (its first-seen copy in sym),
 * out_wcount its multiplicity, *out_n (device int64) the number of distinct words.
 * Output order is unspecified (training results do not depend on it).  Words of 0 or 1
 * symbols are dropped (they hold no pair). out_* sized n_words.
 * Workspace: beast_bpe_dedup_workspace_bytes(n) sizes the hash table for n / 4 distinct words
 * (trajectory corpora repeat their words; K5 is 13 % distinct, and the smaller table stays in the
 * 256 MB Infinity Cache).  With more distinct words than that table holds the call still returns
 * BEAST_OK but writes *out_n = -1 (the outputs are then undefined): retry with a larger workspace
 * (the in-tree callers multiply it by 4).  beast_bpe_dedup_workspace_bytes_safe(n) sizes a table
 * of >= 2 n slots, which can never fill: with it *out_n is always the distinct count. */
size_t beast_bpe_dedup_workspace_bytes(int64_t n_words);
size_t beast_bpe_dedup_workspace_bytes_safe(int64_t n_words);
int beast_bpe_dedup_words(const uint16_t* sym, const uint32_t* wstart, const uint32_t* wlen, int64_t n_words,
                          void* workspace, size_t ws_bytes, uint32_t* out_wstart, uint32_t* out_wlen,
                          uint32_t* out_wcount, int64_t* out_n, void* stream);
/* One-pass setup (round 5): beast_bpe_pretok_count / _emit and beast_bpe_dedup_words fused.
 * Every sequence is pre-tokenised (one wave each, as beast_bpe_pretok_emit) and its words of >= 2
 * byte symbols go straight into the distinct-word table, identified by their code points (a
 * match is confirmed against the first occurrence in `tok` itself); no per-occurrence symbol
 * array is written.  out_info (device int64[4]): distinct words, words, byte symbols, flags --
 * bit 0: the table filled up (retry with 4x the workspace), bit 1: a row the one-pass kernel does
 * not take (over 512 code points, a code point outside [0, 2^31), token offsets from 2^32): run
 * the two-pass functions above instead.  Workspace: beast_bpe_pretok_dedup_workspace_bytes(total
 * tokens; 28 bytes a table slot); it keeps the distinct-word list for beast_bpe_pretok_dedup_repack, which writes the
 * same outputs as beast_bpe_dedup_words + beast_bpe_repack_words (words of >= 2 symbols in
 * length order, their counts), byte symbols made from the code points (byte2id as pretok_emit).
 * repack_ws_bytes >= beast_bpe_repack_workspace_bytes(n_distinct) + 8 * (n_distinct + 1). */
size_t beast_bpe_pretok_dedup_workspace_bytes(int64_t n_tokens);
int beast_bpe_pretok_dedup(const int64_t* tok, const int64_t* seq_off, int64_t n_seq, int64_t min_tok,
                           const uint8_t* cls_lut, int64_t lut_n, void* workspace, size_t ws_bytes, int64_t* out_info,
                           void* stream);
int beast_bpe_pretok_dedup_repack(const int64_t* tok, int64_t min_tok, const uint16_t* byte2id, void* workspace,
                                  size_t ws_bytes, int64_t n_distinct, void* repack_ws, size_t repack_ws_bytes,
                                  uint16_t* out_sym, uint32_t* out_wstart, uint32_t* out_wlen, uint32_t* out_wcount,
                                  int64_t* out_nsym, void* stream);
/* Copy words into one symbol array ordered by length (min(L, 255) buckets, order inside a
 * bucket unspecified); each word starts at a multiple of 4 symbols (8 bytes) and owns its length
 * rounded up to 4 (the padding is zero): the layout the merge loops read and write in 8-byte
 * units.  out_sym capacity >= sum of round_up(wlen, 4); *out_nsym (device int64) = symbols of
 * the padded layout.  wcount may be NULL. */
size_t beast_bpe_repack_workspace_bytes(int64_t n_words);
int beast_bpe_repack_words(const uint16_t* sym, const uint32_t* wstart, const uint32_t* wlen, const uint32_t* wcount,
                           int64_t n_words, void* workspace, size_t ws_bytes, uint16_t* out_sym,
                           uint32_t* out_wstart, uint32_t* out_wlen, uint32_t* out_wcount, int64_t* out_nsym,
                           void* stream);
/* Keep the words that still have >= 2 symbols (order unspecified); *out_n device int64.
 * wcount may be NULL (count 1). */
int beast_bpe_compact_words(const uint32_t* wstart, const uint32_t* wlen, const uint32_t* wcount, int64_t n_words,
                            uint32_t* out_wstart, uint32_t* out_wlen, uint32_t* out_wcount, int64_t* out_n,
                            void* stream);

/* ------------------------------------------------------- §8f rank 1: BPE codec ---
 * Per-row BPE inference with a trained byte-level model, replacing
 * beast/beast_bspline_bpe_tokenizer.py:175-198 (_discrete_to_bpe: per row
 * tokenizer.encode("".join(map(chr, row - min)), add_special_tokens=False).ids) and
 * :200-247 (_bpe_to_discrete: tokenizer.decode(ids, skip_special_tokens=True), ord + min).
 * HF tokenizers semantics: AddedVocabulary split on special tokens (leftmost-longest),
 * ByteLevel pre-tokeniser, BPE::merge_word / Word::merge_all (rank, pos) min-heap,
 * ByteLevel decoder + String::from_utf8_lossy.
 *
 * Merge map: (a, b) -> (rank, new_id), open addressing in device memory; merges in rank
 * order (a pair listed twice keeps its last rank, as HF's HashMap collect). ids < 65536. */
int beast_bpe_mergemap_log2cap(int n_merges);
size_t beast_bpe_mergemap_bytes(int n_merges);
int beast_bpe_mergemap_build(const int32_t* merge_a, const int32_t* merge_b, const int32_t* merge_new,
                             int n_merges, void* map, size_t map_bytes, void* stream);
/* Encode rows tok[row_off[r] .. row_off[r+1]) (int64 bins).  Shifted code point
 * v = tok - min_tok; status[r]: 0 ok, 1 some v < 0, 2 some v > max_span (max_span >= 0),
 * 3 v > 0x10FFFF, 4 surrogate, 5 v >= lut_n (no class), 6 row longer than max_row_cps /
 * max_row_syms.  byte2id[256]: vocab id of each byte-level char, -1 if absent (dropped, or
 * unk_id (fused when fuse_unk) if the model has an unk token).  Special tokens:
 * spec_cps[n_spec][64] code points, spec_len, spec_id.  Output: out_ids[r][0 .. out_len[r])
 * (row stride out_stride >= max_row_syms).  LDS per row: beast_bpe_encode_lds_bytes (one row
 * must fit 160 KiB, else BEAST_E_UNSUPPORTED); a workgroup holds the merge map once (when it
 * fits beside a row) and as many rows as fit, up to 16. */
size_t beast_bpe_encode_lds_bytes(int max_row_cps, int max_row_syms);
int beast_bpe_encode_rows(const int64_t* tok, const int64_t* row_off, int64_t n_rows, int64_t min_tok,
                          int64_t max_span, const uint8_t* cls_lut, int64_t lut_n, const int32_t* byte2id,
                          const void* map, int n_merges, const int32_t* spec_cps, const int32_t* spec_len,
                          const int32_t* spec_id, int n_spec, int unk_id, int fuse_unk, int max_row_cps,
                          int max_row_syms, int32_t* out_ids, int64_t out_stride, int32_t* out_len,
                          int32_t* status, void* stream);
/* The same encode by words (round 4), one launch, no workspace: each workgroup pre-tokenises
 * its rows (up to 16), merges every distinct word among them once (exact dedup by code points in
 * LDS) and gathers each row's ids.  Bit-exact with beast_bpe_encode_rows for models whose merges
 * only combine tokens made by earlier merges -- every trained model; the caller checks and uses
 * beast_bpe_encode_rows otherwise, or when the model has special tokens.  status as above plus
 * 7 (ST_FALLBACK): the row holds a word of more than 64 byte symbols; the caller re-encodes such
 * rows with beast_bpe_encode_rows.
 * wordmap: the merges as a two-choice bucketed cuckoo table of 1 << wordmap_log2b buckets,
 * built on the host by beast_bpe_wordmap_build_host into a buffer of beast_bpe_wordmap_bytes
 * (HOST pointers; it returns the bucket count's log2) and copied to the device (its first
 * 16 << log2b bytes). */
int beast_bpe_wordmap_log2buckets(int n_merges);
size_t beast_bpe_wordmap_bytes(int n_merges);
int beast_bpe_wordmap_build_host(const int32_t* host_merge_a, const int32_t* host_merge_b,
                                 const int32_t* host_merge_new, int n_merges, void* host_out, size_t bytes,
                                 int* host_log2b_out);
int beast_bpe_encode_rows_words(const int64_t* tok, const int64_t* row_off, int64_t n_rows, int64_t min_tok,
                                int64_t max_span, const uint8_t* cls_lut, int64_t lut_n, const int32_t* byte2id,
                                const void* wordmap, int wordmap_log2b, int unk_id, int fuse_unk, int max_row_cps,
                                int max_row_syms, int32_t* out_ids, int64_t out_stride, int32_t* out_len,
                                int32_t* status, void* stream);
/* Decode rows ids[row_off[r] .. row_off[r+1]).  tok_off[n_vocab+1] / tok_bytes: each id's
 * ByteLevel-decoded bytes; tok_skip[id] = 1 for special tokens (skip_special_tokens) and
 * unassigned ids.  out[r][0 .. min(count, L)) = code point + min_tok; out_count[r] = code
 * points decoded (the caller checks == L); status[r] bit 0: the row holds unk_id, bit 1: it
 * holds an id < -1 (the caller's mark for a value that is not a u32).  Id -1 is skipped. */
int beast_bpe_decode_rows(const int32_t* ids, const int64_t* row_off, int64_t n_rows, const int32_t* tok_off,
                          const uint8_t* tok_bytes, const uint8_t* tok_skip, int n_vocab, int unk_id,
                          int64_t min_tok, int L, int64_t* out, int32_t* out_count, int32_t* status,
                          void* stream);

#ifdef __cplusplus
}
#endif
#endif /* BEAST_HIP_H */
