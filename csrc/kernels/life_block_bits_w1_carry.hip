// life_block variant: BitsIO<1, kXlaneCarry> (see life_block_impl.hpp).
#include "life_block_launch.hpp"

namespace gol {
namespace hipk {

GOL_LIFE_VARIANT(launch_bits_w1_carry) { lb::launch_variant<lb::BitsIO<1, kXlaneCarry>>(p, out_rows, T, tune, s); }

}  // namespace hipk
}  // namespace gol
