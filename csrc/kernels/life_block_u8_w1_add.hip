// life_block variant: U8IO<1, kXlaneAdd> (see life_block_impl.hpp): the
// one-sided add-with-carry window, no cross-lane data ops.
#include "life_block_launch.hpp"


namespace gol {
namespace hipk {

GOL_LIFE_VARIANT(launch_u8_w1_add) { lb::launch_variant<lb::U8IO<1, kXlaneAdd>>(p, out_rows, T, tune, s); }

}  // namespace hipk
}  // namespace gol
