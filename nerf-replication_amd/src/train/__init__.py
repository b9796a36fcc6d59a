from .optimizer import make_optimizer  # noqa: F401
from .recorder import make_recorder  # noqa: F401
from .scheduler import make_lr_scheduler, set_lr_scheduler  # noqa: F401
from .trainers import make_trainer  # noqa: F401
