// Resident epoch kernel instantiations (life_resident_impl.hpp): rows per wave 8, 9, 10, 11, 12, 13.
#include "life_resident_impl.hpp"

GOL_RESIDENT_RW(8)
GOL_RESIDENT_RW(9)
GOL_RESIDENT_RW(10)
GOL_RESIDENT_RW(11)
GOL_RESIDENT_RW(12)
GOL_RESIDENT_RW(13)
