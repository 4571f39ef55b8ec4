// Resident epoch kernel instantiations (life_resident_impl.hpp): rows per wave 8, 10, 12, 14.
#include "life_resident_impl.hpp"

GOL_RESIDENT_RW(8)
GOL_RESIDENT_RW(10)
GOL_RESIDENT_RW(12)
GOL_RESIDENT_RW(14)
