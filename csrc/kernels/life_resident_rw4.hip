// Resident epoch kernel instantiations (life_resident_impl.hpp): rows per wave 40, 44, 48, 52.
#include "life_resident_impl.hpp"

GOL_RESIDENT_RW(40)
GOL_RESIDENT_RW(44)
GOL_RESIDENT_RW(48)
GOL_RESIDENT_RW(52)
