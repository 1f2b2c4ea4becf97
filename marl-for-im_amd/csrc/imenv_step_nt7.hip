// Step kernel instantiations for node capacity 7 (see imenv_step_inst.h).
#define IMENV_NT 7
#include "imenv_step_inst.h"
