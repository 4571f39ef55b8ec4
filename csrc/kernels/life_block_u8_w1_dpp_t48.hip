// T = 48 byte-layout passes of the U8IO<1, kXlaneDpp> variant: level-pipelined
// wave pairs of 24 + 24 levels (life_block_launch.hpp launch_deep_pipe), in a
// translation unit of their own.
#include "life_block_launch.hpp"

GOL_U8_PIPE(, 24, 24, kXlaneDpp)
