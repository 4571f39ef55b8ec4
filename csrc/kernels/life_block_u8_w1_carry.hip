// life_block variant: U8IO<1, kXlaneCarry> (see life_block_impl.hpp).
#include "life_block_launch.hpp"

GOL_U8_DEEP(extern, 24, kXlaneCarry)
GOL_U8_DEEP(extern, 32, kXlaneCarry)

namespace gol {
namespace hipk {

GOL_LIFE_VARIANT(launch_u8_w1_carry) { lb::launch_variant<lb::U8IO<1, kXlaneCarry>>(p, out_rows, T, tune, s); }

}  // namespace hipk
}  // namespace gol
