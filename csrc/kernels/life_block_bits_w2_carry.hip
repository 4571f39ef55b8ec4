// life_block variant: BitsIO<2, kXlaneCarry> (see life_block_impl.hpp).
#include "life_block_launch.hpp"

namespace gol {
namespace hipk {

GOL_LIFE_VARIANT(launch_bits_w2_carry) { lb::launch_variant<lb::BitsIO<2, kXlaneCarry>>(p, out_rows, T, tune, s); }

}  // namespace hipk
}  // namespace gol
