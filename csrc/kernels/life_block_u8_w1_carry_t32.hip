// T = 32 byte-layout passes of the U8IO<1, kXlaneCarry> variant
// (life_block_launch.hpp launch_deep), in a translation unit of their own.
#include "life_block_launch.hpp"

GOL_U8_DEEP(, 32, kXlaneCarry)
