// lqrx_kkt.hip — batched block-tridiagonal KKT solve (placeholder launcher, filled below).
#include "lqrx_internal.h"
namespace lqrx {
hipError_t kkt_launch(const KktArgs &, hipStream_t) { return hipErrorNotSupported; }
}
