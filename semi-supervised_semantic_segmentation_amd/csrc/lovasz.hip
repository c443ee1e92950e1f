// Binary Lovász-softmax (losses.py:239-250 -> lovasz.py:155-201, lovasz_grad lovasz.py:19-31).
// Placeholder entry points: the segmented radix sort lands in a later milestone.  Until then the
// calls fail loudly (SSSEG_EUNSUPPORTED) so nothing silently falls back to a CPU path.
#include "common.h"

extern "C" size_t ssseg_lovasz_workspace_bytes(int64_t B, int64_t HW) { return (size_t)(B * HW) * 16 + 4096; }

extern "C" int ssseg_lovasz_fwd(const float*, const float*, int64_t, int64_t, int64_t, float*, void*, size_t,
                                ssseg_stream_t) {
  return SSSEG_EUNSUPPORTED;
}

extern "C" int ssseg_lovasz_bwd(const float*, const float*, int64_t, int64_t, int64_t, const float*, float*, void*,
                                size_t, ssseg_stream_t) {
  return SSSEG_EUNSUPPORTED;
}
