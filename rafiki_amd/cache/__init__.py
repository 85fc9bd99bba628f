from .cache import Cache
from .mq import MessageQueue

__all__ = ['Cache', 'MessageQueue']
