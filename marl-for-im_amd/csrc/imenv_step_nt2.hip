// Step kernel instantiations for node capacity 2 (see imenv_step_inst.h).
#define IMENV_NT 2
#include "imenv_step_inst.h"
