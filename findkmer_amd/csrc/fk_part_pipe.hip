/* fk_part_*.hip -- k_part instances (fk_part_kern.h): the pipelined main passes (k = 8..13) */
#include "fk_part_kern.h"

FK_PART_PIPE_INSTANCES(FK_PART_INSTANTIATE)
