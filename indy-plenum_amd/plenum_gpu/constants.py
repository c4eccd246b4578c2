"""Field names used on the authentication path (plenum/common/types.py:27-88,
plenum/common/constants.py:77-154)."""
IDENTIFIER = 'identifier'
SIGNATURE = 'signature'
SIGNATURES = 'signatures'
FEES = 'fees'
OPERATION = 'operation'
TXN_TYPE = 'type'
VERKEY = 'verkey'
ROLE = 'role'
TARGET_NYM = 'dest'
NYM = '1'
