// Resident epoch kernel instantiations (life_resident_impl.hpp): rows per wave 56, 60, 64, 72.
#include "life_resident_impl.hpp"

GOL_RESIDENT_RW(56)
GOL_RESIDENT_RW(60)
GOL_RESIDENT_RW(64)
GOL_RESIDENT_RW(72)
