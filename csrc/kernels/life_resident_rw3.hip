// Resident epoch kernel instantiations (life_resident_impl.hpp): rows per wave 26, 27, 28, 29, 30, 31.
#include "life_resident_impl.hpp"

GOL_RESIDENT_RW(26)
GOL_RESIDENT_RW(27)
GOL_RESIDENT_RW(28)
GOL_RESIDENT_RW(29)
GOL_RESIDENT_RW(30)
GOL_RESIDENT_RW(31)
