// Step kernel instantiations for node capacity 3 (see imenv_step_inst.h).
#define IMENV_NT 3
#include "imenv_step_inst.h"
