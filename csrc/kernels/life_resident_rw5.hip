// Resident epoch kernel instantiations (life_resident_impl.hpp): rows per wave 38, 39, 40, 41, 42, 43.
#include "life_resident_impl.hpp"

GOL_RESIDENT_RW(38)
GOL_RESIDENT_RW(39)
GOL_RESIDENT_RW(40)
GOL_RESIDENT_RW(41)
GOL_RESIDENT_RW(42)
GOL_RESIDENT_RW(43)
