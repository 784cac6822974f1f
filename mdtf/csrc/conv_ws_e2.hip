// Weight-stationary conv kernels, epilogue mode 2 (see conv_ws_kernel.inc / conv_ws.hip).
#include "conv_ws_kernel.inc"

namespace mdtf {
namespace ws {
template int dispatch_ws<2>(WsArgs&, int, int, int, int, int, hipStream_t);
}  // namespace ws
}  // namespace mdtf
