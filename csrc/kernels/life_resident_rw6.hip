// Resident epoch kernel instantiations (life_resident_impl.hpp): rows per wave 44, 45, 46, 47, 48, 52.
#include "life_resident_impl.hpp"

GOL_RESIDENT_RW(44)
GOL_RESIDENT_RW(45)
GOL_RESIDENT_RW(46)
GOL_RESIDENT_RW(47)
GOL_RESIDENT_RW(48)
GOL_RESIDENT_RW(52)
