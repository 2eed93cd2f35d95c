/* CPU oracle for the index-finalize arrays — TEST INFRASTRUCTURE ONLY.
 *
 * Restates, step for step, what the reference's IndexBuilder writes besides the MPHF
 * (SURVEY.md §8 row f4):
 *   - depth.u32: row.Depth per prefix in Add order (indexbuild.go:185); the aggregator
 *     sets Depth = number of '/' in the prefix ("" -> 0, "a/" -> 1; aggregator.go:44-60);
 *   - subtree_end.u64 / max_depth_in_subtree.u32: the ancestor stack of
 *     indexbuild.go:154-248 (findCommonAncestorDepth: the leading stack entries that are
 *     byte prefixes of the new prefix; closeNodesAbove / closeTopNode: a popped node's
 *     subtree ends at the last position added so far and its max depth propagates to its
 *     parent); Finalize closes the rest (:393-395) and writes both arrays (:474-503);
 *   - depth_offsets.u64 / depth_positions.u64: DepthIndexBuilder.Build
 *     (depthindex.go:32-96): for d = 0..maxDepth the offset, then that depth's positions
 *     ascending, then the sentinel offset — maxDepth + 2 offsets.
 * Only tests/ may load this; the product computes the same arrays on the GPU.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
  uint64_t pos;
  uint64_t off, len; /* the prefix bytes, for the prefix test */
  uint32_t max_depth;
} orc_stack_entry;

/* depths: caller's row.Depth values, or NULL to count '/' bytes.  Outputs (caller-sized):
 * depth_out[n], subtree_end[n], max_depth_sub[n], depth_positions[n], and depth_offsets
 * with room for off_cap entries; *max_depth_out receives maxDepth.  Returns 0, or -1 if
 * off_cap < maxDepth + 2 (nothing past depth_out is written then), -2 out of memory. */
int orc_finalize(const uint8_t* blob, const uint64_t* offsets, const uint32_t* depths, uint64_t n,
                 uint32_t* depth_out, uint64_t* subtree_end, uint32_t* max_depth_sub, uint64_t* depth_offsets,
                 uint64_t off_cap, uint64_t* depth_positions, uint32_t* max_depth_out) {
  uint32_t maxd = 0;
  for (uint64_t i = 0; i < n; ++i) {
    uint32_t d = 0;
    if (depths) {
      d = depths[i];
    } else {
      for (uint64_t b = offsets[i]; b < offsets[i + 1]; ++b) d += blob[b] == '/';
    }
    depth_out[i] = d;
    if (d > maxd) maxd = d;
  }
  *max_depth_out = maxd;
  if (off_cap < (uint64_t)maxd + 2) return -1;
  /* the ancestor stack (indexbuild.go:154-248) */
  orc_stack_entry* st = (orc_stack_entry*)malloc(sizeof(orc_stack_entry) * (n ? n : 1));
  if (!st) return -2;
  uint64_t top = 0, pos_count = 0;
  for (uint64_t i = 0; i < n; ++i) {
    const uint64_t off = offsets[i], len = offsets[i + 1] - offsets[i];
    uint64_t common = 0;
    for (uint64_t s = 0; s < top; ++s) {
      if (st[s].len <= len && memcmp(blob + st[s].off, blob + off, st[s].len) == 0)
        common = s + 1;
      else
        break;
    }
    while (top > common) { /* closeTopNode */
      const orc_stack_entry e = st[--top];
      subtree_end[e.pos] = pos_count - 1;
      max_depth_sub[e.pos] = e.max_depth;
      if (top && e.max_depth > st[top - 1].max_depth) st[top - 1].max_depth = e.max_depth;
    }
    st[top].pos = pos_count++;
    st[top].off = off;
    st[top].len = len;
    st[top].max_depth = depth_out[i];
    ++top;
  }
  while (top) { /* Finalize: closeNodesAbove(0) */
    const orc_stack_entry e = st[--top];
    subtree_end[e.pos] = pos_count - 1;
    max_depth_sub[e.pos] = e.max_depth;
    if (top && e.max_depth > st[top - 1].max_depth) st[top - 1].max_depth = e.max_depth;
  }
  free(st);
  /* DepthIndexBuilder.Build: positions grouped by depth, ascending within a depth */
  uint64_t* cnt = (uint64_t*)calloc((size_t)maxd + 2, sizeof(uint64_t));
  if (!cnt) return -2;
  for (uint64_t i = 0; i < n; ++i) ++cnt[depth_out[i]];
  uint64_t acc = 0;
  for (uint32_t d = 0; d <= maxd; ++d) {
    depth_offsets[d] = acc;
    acc += cnt[d];
    cnt[d] = depth_offsets[d];
  }
  depth_offsets[maxd + 1] = acc;
  for (uint64_t i = 0; i < n; ++i) depth_positions[cnt[depth_out[i]]++] = i;
  free(cnt);
  return 0;
}
