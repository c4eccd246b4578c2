OBJECT = 'py/object'
STATE = 'py/state'
