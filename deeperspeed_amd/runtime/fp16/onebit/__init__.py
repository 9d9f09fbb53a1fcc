from .adam import OnebitAdam
from .lamb import OnebitLamb
