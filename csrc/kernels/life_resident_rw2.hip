// Resident epoch kernel instantiations (life_resident_impl.hpp): rows per wave 20, 21, 22, 23, 24, 25.
#include "life_resident_impl.hpp"

GOL_RESIDENT_RW(20)
GOL_RESIDENT_RW(21)
GOL_RESIDENT_RW(22)
GOL_RESIDENT_RW(23)
GOL_RESIDENT_RW(24)
GOL_RESIDENT_RW(25)
