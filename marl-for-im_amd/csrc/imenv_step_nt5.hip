// Step kernel instantiations for node capacity 5 (see imenv_step_inst.h).
#define IMENV_NT 5
#include "imenv_step_inst.h"
