// Step kernel instantiations for node capacity 1 (see imenv_step_inst.h).
#define IMENV_NT 1
#include "imenv_step_inst.h"
