// Weight-stationary conv kernels, epilogue mode 5 (see conv_ws_kernel.inc / conv_ws.hip).
#include "conv_ws_kernel.inc"

namespace mdtf {
namespace ws {
template int dispatch_ws<5>(WsArgs&, int, int, int, int, int, hipStream_t);
}  // namespace ws
}  // namespace mdtf
