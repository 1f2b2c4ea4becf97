// Step kernel instantiations for node capacity 4 (see imenv_step_inst.h).
#define IMENV_NT 4
#include "imenv_step_inst.h"
