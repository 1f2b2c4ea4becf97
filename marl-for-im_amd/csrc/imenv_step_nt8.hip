// Step kernel instantiations for node capacity 8 (see imenv_step_inst.h).
#define IMENV_NT 8
#include "imenv_step_inst.h"
