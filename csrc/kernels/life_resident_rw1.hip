// Resident epoch kernel instantiations (life_resident_impl.hpp): rows per wave 14, 15, 16, 17, 18, 19.
#include "life_resident_impl.hpp"

GOL_RESIDENT_RW(14)
GOL_RESIDENT_RW(15)
GOL_RESIDENT_RW(16)
GOL_RESIDENT_RW(17)
GOL_RESIDENT_RW(18)
GOL_RESIDENT_RW(19)
