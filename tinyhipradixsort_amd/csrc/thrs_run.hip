// thrs_run.hip -- one key type's launch sequences (thrs_host.hpp run_sort),
// compiled once per key type: -DTHRS_RUN_KT=0..3 (U32, U64, F32, F64).
#include "thrs_host.hpp"

namespace thrs_host {
template int run_vb<THRS_RUN_KT>(int, void*, void*, uint32_t, void*, void*, void*, int, int, bool, const Plan&,
                                 const thrs_options&, hipStream_t, uint32_t*);
}  // namespace thrs_host
