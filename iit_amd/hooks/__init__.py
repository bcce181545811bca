from .hook_points import ActivationCache, HookedRootModule, HookPoint, get_act_name
from .wrapper import HookedModuleWrapper, get_hook_points
