// Resident epoch kernel instantiations (life_resident_impl.hpp): rows per wave 32, 34, 36, 38.
#include "life_resident_impl.hpp"

GOL_RESIDENT_RW(32)
GOL_RESIDENT_RW(34)
GOL_RESIDENT_RW(36)
GOL_RESIDENT_RW(38)
