/* fk_part_*.hip -- k_part instances (fk_part_kern.h): the phase-by-phase main passes (k = 14..16) and every k_part<RES> */
#include "fk_part_kern.h"

FK_PART_OTHER_INSTANCES(FK_PART_INSTANTIATE)
