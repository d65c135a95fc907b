/*
 * jansson.h — the subset of the jansson 2.x API that the NAV-SLAM driver
 * (src/main.c:3,13-74,131-185) calls, so the reference main.c compiles and
 * links unchanged in an image without jansson.
 *
 * Implemented by jansson_mini.c. Semantics follow jansson's documented
 * behaviour for exactly these calls:
 *   - a JSON number without '.', 'e' or 'E' is an integer (json_int_t = long
 *     long), anything else a real parsed with strtod;
 *   - json_integer_value() of a non-integer and json_real_value() of a
 *     non-real return 0 -- so an IMU "params" entry written as `1` (no decimal
 *     point) reads as 0.0 in main.c:171-176, as with the real library;
 *   - json_is_*() of NULL is false; json_object_get() of a non-object or of a
 *     missing key is NULL; json_array_get() out of range is NULL; a repeated
 *     object key keeps its last value;
 *   - json_loadf() parses the rest of the stream as one JSON text whose top
 *     level is an array or an object (jansson without JSON_DECODE_ANY; other
 *     flags are ignored) and returns NULL with error->text set on any error.
 * Nothing outside this list is provided.
 */
#ifndef NAVSLAM_JANSSON_MINI_H
#define NAVSLAM_JANSSON_MINI_H

#include <stddef.h>
#include <stdio.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef long long json_int_t;

typedef enum {
    JSON_OBJECT,
    JSON_ARRAY,
    JSON_STRING,
    JSON_INTEGER,
    JSON_REAL,
    JSON_TRUE,
    JSON_FALSE,
    JSON_NULL
} json_type;

typedef struct json_t {
    json_type type;
    size_t refcount;
} json_t;

#define JSON_ERROR_TEXT_LENGTH 160
#define JSON_ERROR_SOURCE_LENGTH 80

typedef struct json_error_t {
    int line;
    int column;
    int position;
    char source[JSON_ERROR_SOURCE_LENGTH];
    char text[JSON_ERROR_TEXT_LENGTH];
} json_error_t;

#define json_typeof(json) ((json)->type)
#define json_is_object(json) ((json) && json_typeof(json) == JSON_OBJECT)
#define json_is_array(json) ((json) && json_typeof(json) == JSON_ARRAY)
#define json_is_string(json) ((json) && json_typeof(json) == JSON_STRING)
#define json_is_integer(json) ((json) && json_typeof(json) == JSON_INTEGER)
#define json_is_real(json) ((json) && json_typeof(json) == JSON_REAL)
#define json_is_number(json) (json_is_integer(json) || json_is_real(json))

json_t *json_loadf(FILE *input, size_t flags, json_error_t *error);
json_t *json_loads(const char *input, size_t flags, json_error_t *error);
void json_delete(json_t *json);

/* true/false/null are shared singletons (refcount (size_t)-1, never freed) */
static inline void json_decref(json_t *json) {
    if (json && json->refcount != (size_t)-1 && --json->refcount == 0)
        json_delete(json);
}

size_t json_array_size(const json_t *array);
json_t *json_array_get(const json_t *array, size_t index);
json_t *json_object_get(const json_t *object, const char *key);
json_int_t json_integer_value(const json_t *integer);
double json_real_value(const json_t *real);
const char *json_string_value(const json_t *string);

#define json_array_foreach(array, index, value)                                \
    for (index = 0;                                                            \
         index < json_array_size(array) && (value = json_array_get(array, index)); \
         index++)

#ifdef __cplusplus
}
#endif
#endif
