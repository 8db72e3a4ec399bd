// Host-side ragged batch metadata for the inference-v2 (FastGen + HCache) engine, built in one pass into ONE
// int32 buffer (pinned by the caller) so a forward ships its whole batch description with a single H2D copy.
//
// Capability parity: reference inference/v2/ragged/csrc/ragged_ops.cpp (`RaggedBatchWrapper` finalize: the
// inflight sequence descriptors, token -> sequence map, KV block table) and
// inference/v2/kernels/ragged_ops/atom_builder/atom_builder.cpp:10-52 (`build_atoms`: one attention work item per
// (sequence, kv head, query-row chunk)). The reference runs them per forward in C++ for exactly the reason the
// Python versions were slow here: a decode step of B sequences is O(B * n_kv) small items per layer-forward.
//
// Layout of `out` (int32), S = n_seqs, T = sum(n_new), A = atoms:
//   [0, 3S)                 seq_meta  (q_start, n_new, seen) per sequence
//   [3S, 3S+T)              tok_seq   sequence index of every token
//   [3S+T, 3S+2T)           tok_pos   absolute position of every token (seen + i)
//   [3S+2T, 4S+2T)          last      index of each sequence's last token (logits rows)
//   [4S+2T, 4S+2T+S*MB)     tables    KV block ids per sequence, MB = max_blocks columns, zero padded
//   [..., + 3A)             atoms     (seq, kv_head, row_start) with rows = n_new * (n_q / n_kv) per (seq, kv head)
// Returns A, or -1 when `cap` is too small (the required size is then written to *need).
#include <cstdint>
#include <cstring>

#define HDS_EXPORT extern "C" __attribute__((visibility("default")))

HDS_EXPORT int64_t hds_ragged_meta_size(int n_seqs, int64_t n_tokens, int max_blocks, int64_t n_atoms) {
  return 4LL * n_seqs + 2LL * n_tokens + (int64_t)n_seqs * max_blocks + 3LL * n_atoms;
}

HDS_EXPORT int64_t hds_ragged_meta_build(const int32_t* n_new, const int32_t* seen, int n_seqs,
                                         const int32_t* blocks, const int64_t* block_off, int max_blocks, int n_q,
                                         int n_kv, int rows_per_atom, int32_t* out, int64_t cap, int64_t* need) {
  if (n_seqs < 0 || n_kv <= 0 || n_q % n_kv != 0 || rows_per_atom <= 0 || max_blocks < 0) return -2;
  const int G = n_q / n_kv;
  int64_t T = 0, A = 0;
  for (int s = 0; s < n_seqs; ++s) {
    T += n_new[s];
    const int64_t rows = (int64_t)n_new[s] * G;
    A += (int64_t)n_kv * ((rows + rows_per_atom - 1) / rows_per_atom);
  }
  const int64_t size = hds_ragged_meta_size(n_seqs, T, max_blocks, A);
  if (need) *need = size;
  if (size > cap) return -1;
  int32_t* meta = out;
  int32_t* tok_seq = meta + 3LL * n_seqs;
  int32_t* tok_pos = tok_seq + T;
  int32_t* last = tok_pos + T;
  int32_t* tables = last + n_seqs;
  int32_t* atoms = tables + (int64_t)n_seqs * max_blocks;
  int64_t q0 = 0, a = 0;
  for (int s = 0; s < n_seqs; ++s) {
    const int32_t n = n_new[s], sn = seen[s];
    meta[3 * s] = (int32_t)q0;
    meta[3 * s + 1] = n;
    meta[3 * s + 2] = sn;
    for (int32_t i = 0; i < n; ++i) {
      tok_seq[q0 + i] = s;
      tok_pos[q0 + i] = sn + i;
    }
    last[s] = (int32_t)(q0 + (n > 0 ? n - 1 : 0));
    const int64_t b0 = block_off[s], nb = block_off[s + 1] - b0;
    int32_t* row = tables + (int64_t)s * max_blocks;
    const int64_t ncopy = nb < max_blocks ? nb : max_blocks;
    if (ncopy > 0) std::memcpy(row, blocks + b0, sizeof(int32_t) * ncopy);
    if (ncopy < max_blocks) std::memset(row + ncopy, 0, sizeof(int32_t) * (max_blocks - ncopy));
    const int64_t rows = (int64_t)n * G;
    for (int hk = 0; hk < n_kv; ++hk)
      for (int64_t r0 = 0; r0 < rows; r0 += rows_per_atom) {
        atoms[3 * a] = s;
        atoms[3 * a + 1] = hk;
        atoms[3 * a + 2] = (int32_t)r0;
        ++a;
      }
    q0 += n;
  }
  return A;
}
