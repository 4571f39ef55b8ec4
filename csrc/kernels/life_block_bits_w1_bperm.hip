// life_block variant: BitsIO<1, kXlaneBpermute> (see life_block_impl.hpp).
#include "life_block_launch.hpp"

namespace gol {
namespace hipk {

GOL_LIFE_VARIANT(launch_bits_w1_bperm) { lb::launch_variant<lb::BitsIO<1, kXlaneBpermute>>(p, out_rows, T, tune, s); }

}  // namespace hipk
}  // namespace gol
