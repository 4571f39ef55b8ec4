// life_block variant: U8IO<1, kXlaneDpp> (see life_block_impl.hpp).
#include "life_block_launch.hpp"

GOL_U8_DEEP(extern, 24, kXlaneDpp)
GOL_U8_DEEP(extern, 32, kXlaneDpp)

namespace gol {
namespace hipk {

GOL_LIFE_VARIANT(launch_u8_w1_dpp) { lb::launch_variant<lb::U8IO<1, kXlaneDpp>>(p, out_rows, T, tune, s); }

}  // namespace hipk
}  // namespace gol
