// Resident epoch kernel instantiations (life_resident_impl.hpp): rows per wave 32, 33, 34, 35, 36, 37.
#include "life_resident_impl.hpp"

GOL_RESIDENT_RW(32)
GOL_RESIDENT_RW(33)
GOL_RESIDENT_RW(34)
GOL_RESIDENT_RW(35)
GOL_RESIDENT_RW(36)
GOL_RESIDENT_RW(37)
