// Flow launches (life_flow_impl.hpp), bit layout, symmetric DPP window:
// T = 8, 12 and 16, 4- and 8-wave items.
#include "life_flow_impl.hpp"

namespace gol {
namespace hipk {

GOL_FLOW_VARIANT(launch_flow_bits_dpp) {
  using IO = lb::BitsIO<1, kXlaneDpp>;
  switch (T) {
    case 8: return lb::launch_flow_T<8, IO>(f, rows_min, tune, s, desc, tickets, items);
    case 12: return lb::launch_flow_T<12, IO>(f, rows_min, tune, s, desc, tickets, items);
    case 16: return lb::launch_flow_T<16, IO>(f, rows_min, tune, s, desc, tickets, items);
    default: return false;
  }
}

}  // namespace hipk
}  // namespace gol
